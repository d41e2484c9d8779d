#!/bin/bash
# round-5 GPU call 58: with the wave-uniform conv1 weights: the new library-forward split-plan test, the multistream /
# bit-exact plan tests, and the round-3 xfail (2 ranks sharing the card, the same DP plan twice) 6 times
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_flagship_gpu.py -m gpu -x -v -k "library_fc_forward or multistream or bit_exact_over_12" --timeout 200 --timeout-method thread > $O/r5_58_pytest.log 2>&1 || { tail -30 $O/r5_58_pytest.log; exit 1; }
grep -c PASSED $O/r5_58_pytest.log; tail -1 $O/r5_58_pytest.log
for i in 1 2 3 4 5 6; do
  timeout -k 10 300 python -u -m pytest tests/test_flagship_gpu.py -m gpu -x -q -rxX -k "test_dp_plan_run_to_run_on_shared_gpu" --timeout 280 --timeout-method thread > $O/r5_58_shared_$i.log 2>&1; rc=$?
  echo "run $i rc=$rc $(tail -1 $O/r5_58_shared_$i.log)" | tee -a $O/r5_58_shared.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
