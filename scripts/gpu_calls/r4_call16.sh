#!/bin/bash
# round-4 GPU call: 4-stage FC GEMM rings (forward cfg 6 = 192 x 128, wgrad cfg 4 = 128 x 128): numerics, isolated
# timing, in-step A/B against the shipped 1,1,2
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 120 --timeout-method thread -k "fwd or wgrad" > $O/r4_16_pytest.log 2>&1; echo "pytest rc=$?" >> $O/r4_16_pytest.log
PROBE_ONLY=fwd_hand0,fwd_hand1,fwd_hand2_ks2,fwd_hand6_b4,fwd_hipblaslt,wgrad_hand1,wgrad_hand4_b4 timeout -k 10 300 python scripts/probes/probe_gemm.py > $O/r4_16_gemm_probe.txt 2>&1 || exit 1
VARIANTS="N=0|;N=1|--gemm-cfg 6,1,2;N=2|--gemm-cfg 1,4,2;N=3|--gemm-cfg 6,4,2" bash scripts/gpu_calls/r4_ab.sh $O/r4_16_ab.txt || exit 1
