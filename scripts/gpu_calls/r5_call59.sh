#!/bin/bash
# round-5 GPU call 59: with the wave-uniform conv1 weights:
# the round-3 xfail (2 ranks sharing the card, the same DP plan twice) 14 more times
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
for i in $(seq 1 14); do
  timeout -k 10 300 python -u -m pytest tests/test_flagship_gpu.py -m gpu -x -q -rxX -k "test_dp_plan_run_to_run_on_shared_gpu" --timeout 280 --timeout-method thread > $O/r5_59_shared_$i.log 2>&1; rc=$?
  echo "run $i rc=$rc $(tail -1 $O/r5_59_shared_$i.log)" | tee -a $O/r5_59_shared.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
