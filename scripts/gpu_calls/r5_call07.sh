#!/bin/bash
# round-5 GPU call 7: layer 3's BN backward reduction in the FC data gradient's epilogue (the round-4 wip branch,
# merged, on the producer-wave dgrad tile): conv / flagship / LDS-poison tests, then the step A/B (on / off), and the
# fp8 estimator with e4m3 convs re-measured (verdict r4 item 7)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_flagship_gpu.py tests/test_lds_poison_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r5_07_pytest.log 2>&1 || { tail -40 $O/r5_07_pytest.log; exit 1; }
tail -2 $O/r5_07_pytest.log
for r in 1 2 3; do
  for v in "--knob dgrad_bnred=1" "--knob dgrad_bnred=0"; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 $v > $O/r5_07_cur.json 2> $O/r5_07_cur.err || { tail -20 $O/r5_07_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_07_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_07_ab.txt
  done
done
for r in 1 2; do
  for v in "--dtype fp8" "--dtype fp8 --knob fp8_conv=1"; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 $v > $O/r5_07_cur.json 2> $O/r5_07_cur.err || { tail -20 $O/r5_07_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_07_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_07_fp8.txt
  done
done
