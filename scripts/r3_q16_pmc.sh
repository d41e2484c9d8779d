#!/bin/bash
# PMC passes over the 16-qubit step (one rocprofv3 run per counter set; summaries -> gpurun_out/q16_pmc.md)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
i=0
for pc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
          "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
          "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $pc --output-format csv -d "$OUT/q16pmc_$i" -o run -- python "$ROOT/bench.py" --steps 2 --warmup 1 --settle-steps 0 --steps-per-graph 1 --qubits 16 > "$OUT/q16pmc_$i.log" 2>&1) || { echo "pmc pass $i failed"; tail -5 "$OUT/q16pmc_$i.log"; exit 1; }
done
python "$ROOT/scripts/pmc_summary.py" "$OUT"/q16pmc_* > "$OUT/q16_pmc.md"
rm -rf "$OUT"/q16pmc_*/
