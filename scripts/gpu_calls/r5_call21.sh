#!/bin/bash
# round-5 GPU call 21: layer 3's BN backward reduction in the fp8 estimator's e4m3 data gradient (gemm.hip
# qd_gemm_dgrad_f8_bnred; r5_20's fp8 timeline still ran bn_bwd_reduce on the chain) -- the bnred / fp8 tests, then
# the fp8 step A/B (epilogue vs own launch), 3 alternating rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q -k "bn_reduction or fp8" --timeout 200 --timeout-method thread > $O/r5_21_pytest.log 2>&1 || { tail -40 $O/r5_21_pytest.log; exit 1; }
tail -1 $O/r5_21_pytest.log
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_21_cur.json 2> $O/r5_21_cur.err || { tail -20 $O/r5_21_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_21_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_21_ab.txt
}
for r in 1 2 3; do
  run "r$r fp8 dgrad_bnred" --dtype fp8
  run "r$r fp8 own_launch" --dtype fp8 --knob dgrad_bnred=0
done
