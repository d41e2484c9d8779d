#!/bin/bash
# (1) conv epilogue statistics on v_dot2c_f32_bf16: conv tests + A/B vs the committed library;
# (2) the FC weight's Adam in the wgrad GEMM's epilogue, re-measured with the round-4 plan (plan probe)
cd "$(dirname "$0")/../.." || exit 1
O=$(pwd)/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r4_32_pytest.log 2>&1 || exit 1
bash scripts/ab_lib.sh r4_32 3 || exit 1
PLAN=shipped,fused_adam,fused_adam_w2 ROUNDS=2 timeout -k 10 500 python scripts/probes/r4_plan_probe.py 300 > $O/r4_32_plans.txt 2>&1 || exit 1
