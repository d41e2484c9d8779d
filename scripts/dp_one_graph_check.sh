#!/bin/bash
# One-graph DP plan (RCCL collectives captured) on one GPU: bit-exactness test, then A/B against the
# 5-graph DP plan at world 1 over a real RCCL process group (QDML_FORCE_DIST=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_flagship_gpu.py -m gpu -k one_graph > $OUT/og_test.log 2>&1
rc=$?; tail -5 $OUT/og_test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in "" "--dp-one-graph" "--dp-plan allreduce" "--dp-plan allreduce --dp-one-graph"; do
  QDML_FORCE_DIST=1 timeout -k 10 300 python bench.py --steps 200 --warmup 10 --phase-steps 0 $v > $OUT/og_b.log 2>&1 || { tail -20 $OUT/og_b.log; exit 1; }
  echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/og_b.log)" | tee -a $OUT/og_ab.txt
done; done
