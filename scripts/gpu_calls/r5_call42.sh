#!/bin/bash
# round-5 GPU call 42: "fwd" falls back to the hand plain forward where the loss epilogue does not tile (the tests'
# batch 32 had fallen back to hipBLASLt -- the cause of call 32's split-plan mismatch): full GPU suite, the
# multistream tests with the library forward (expected: the split plans still differ there), step A/B fwd vs fwdplain
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5_42_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/r5_42_pytest.log
tail -3 $O/r5_42_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u -c "
import sys, pytest
from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS
KNOBS.hand_gemm = 'wgrad,dgrad'
sys.exit(pytest.main(['tests/test_flagship_gpu.py', '-q', '-k', 'multistream', '--timeout', '200', '--timeout-method', 'thread', '-p', 'no:cacheprovider']))
" > $O/r5_42_library_fwd.log 2>&1; rc=$?
echo "[library forward] rc=$rc $(tail -1 $O/r5_42_library_fwd.log)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_42_cur.json 2> $O/r5_42_cur.err || { tail -20 $O/r5_42_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_42_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['config']['fc_forward'], d['final_losses'])")" | tee -a $O/r5_42_ab.txt
}
for r in 1 2 3; do
  run "r$r fwd"
  run "r$r fwdplain" --knob hand_gemm=fwdplain,wgrad,dgrad
done
