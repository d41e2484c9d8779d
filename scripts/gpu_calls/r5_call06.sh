#!/bin/bash
# round-5 GPU call 6: the 8-qubit MFMA adjoint (numerics vs the fp64 oracle and qsim.hip's register adjoint), the
# QSC GPU tests on the new default path, and the P128 step A/B (qsim_mfma_bwd on / off), 3 alternating rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qsim12_gpu.py -x -v --timeout 120 --timeout-method thread > $O/r5_06_qsim_pytest.log 2>&1 || { tail -40 $O/r5_06_qsim_pytest.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/r5_06_qsim_pytest.log | tail -20
timeout -k 10 400 python -u -m pytest tests/test_qsc_gpu.py tests/test_flagship_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r5_06_pytest.log 2>&1 || { tail -40 $O/r5_06_pytest.log; exit 1; }
tail -2 $O/r5_06_pytest.log
for r in 1 2 3; do
  for v in "--knob qsim_mfma_bwd=1" "--knob qsim_mfma_bwd=0"; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 $v > $O/r5_06_cur.json 2> $O/r5_06_cur.err || { tail -20 $O/r5_06_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_06_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'], d['config']['qsim_mfma_bwd'])")" | tee -a $O/r5_06_ab.txt
  done
done
