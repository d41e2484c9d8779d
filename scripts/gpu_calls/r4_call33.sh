#!/bin/bash
# layer 3's BN backward reduction in the FC data gradient's epilogue: conv + flagship + gemm tests, A/B against the
# separate reduction launch (plan probe)
cd "$(dirname "$0")/.." || exit 1
O=$(pwd)/gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_conv_gpu.py tests/test_flagship_gpu.py tests/test_gemm_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r4_33_pytest.log 2>&1 || exit 1
PLAN=shipped,no_dgrad_bnred ROUNDS=3 timeout -k 10 500 python scripts/probes/r4_plan_probe.py 300 > $O/r4_33_plans.txt 2>&1 || exit 1
