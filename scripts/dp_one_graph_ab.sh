#!/bin/bash
# world-1 RCCL A/B of the DP plans (QDML_FORCE_DIST=1): 5-graph vs one-graph (1 or 5 steps per replay)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2; do for v in ${VARIANTS:-"|" "|--dp-one-graph --steps-per-graph 5" "|--dp-plan allreduce" "|--dp-plan allreduce --dp-one-graph --steps-per-graph 1" "|--dp-plan allreduce --dp-one-graph --steps-per-graph 5"}; do
  env QDML_FORCE_DIST=1 ${v%%|*} timeout -k 10 300 python bench.py --steps 300 --warmup 10 --phase-steps 0 ${v#*|} > $OUT/og_b.log 2>&1 || { tail -20 $OUT/og_b.log; exit 1; }
  echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/og_b.log)" | tee -a $OUT/og_ab.txt
done; done
