#!/bin/bash
# A/B bench of env-selected variants on one box, alternating, 2 rounds:
#   VARIANTS="A=1|--flags;B=0|" bash scripts/gpu_calls/r4_ab.sh OUTFILE
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
O=${1:-gpurun_out/ab.txt}
IFS=';' read -ra VS <<< "${VARIANTS:-NONE=0|}"
for r in 1 2; do
  for v in "${VS[@]}"; do
    env ${v%%|*} timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 20 ${v#*|} > gpurun_out/ab_cur.json 2> gpurun_out/ab_cur.err || { echo "FAILED $v"; tail -20 gpurun_out/ab_cur.err; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_cur.json)" | tee -a $O
  done
done
