#!/bin/bash
# round-5 GPU call 3: producer-wave GEMM configs -- numerics (test_gemm_gpu.py) and in-step A/B of the FC GEMM
# configs (fwd,wgrad,dgrad) against the shipped 6,1,2, 3 alternating rounds at --steps 300
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r5_03_pytest.log 2>&1 || { tail -30 $O/r5_03_pytest.log; exit 1; }
tail -2 $O/r5_03_pytest.log
for r in 1 2 3; do
  for v in 6,1,2 8,7,6 10,7,6 8,1,2; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 --gemm-cfg $v > $O/r5_03_cur.json 2> $O/r5_03_cur.err || { tail -20 $O/r5_03_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_03_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['config']['fc_gemm_cfg'])")" | tee -a $O/r5_03_ab.txt
  done
done
