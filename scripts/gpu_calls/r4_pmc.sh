#!/bin/bash
# rocprofv3 counter passes over the 1-GPU flagship step (one pass per run, each under its own KILL timeout);
# PASSES: ';'-separated counter lists.  Output: gpurun_out/<tag>_pmc_summary.md
cd "$(dirname "$0")/../.." || exit 1
ROOT=$(pwd)
TAG=${TAG:-pmc}
OUT=$ROOT/gpurun_out
CMD=${CMD:-$ROOT/bench.py --steps 10 --warmup 2 --steps-per-graph 1 --settle-steps 0}
IFS=';' read -ra PS <<< "${PASSES:-FETCH_SIZE}"
i=0
for pc in "${PS[@]}"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $pc --output-format csv -d "$OUT/${TAG}_$i" -o run -- python $CMD > "$OUT/${TAG}_$i.log" 2>&1)
  rc=$?
  echo "pass $i ($pc): rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/${TAG}_$i.log"; exit $rc; fi
done
python scripts/pmc_summary.py "$OUT"/${TAG}_* > "$OUT/${TAG}_pmc_summary.md" && rm -rf "$OUT"/${TAG}_*/
