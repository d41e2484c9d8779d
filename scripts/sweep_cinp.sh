#!/bin/bash
# Conv tile pixel padding sweep (rebuilds the HIP library per value on the GPU box; kernel stats per value).
set -o pipefail
OUT=gpurun_out
for pad in ${PADS:-8 16 24}; do
  QDML_HIPCC_EXTRA="-DQD_CINP_PAD=$pad" timeout -k 10 300 python -c "from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as n; n.build_hip(force=True, verbose=False, jobs=16)" > $OUT/build_$pad.log 2>&1 || exit 1
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/cinp_$pad" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 5 > "$GRAFT_REPO_ROOT/$OUT/cinp_$pad.log" 2>&1) || exit 1
  python scripts/prof_summary.py "$OUT/cinp_$pad/run_kernel_trace.csv" --tail 0.6 > "$OUT/cinp_$pad.md"
  rm -rf "$OUT/cinp_$pad"
done
