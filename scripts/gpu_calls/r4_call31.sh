#!/bin/bash
# the FC weight's Adam in the weight-gradient GEMM's epilogue, re-measured with the round-4 plan
cd "$(dirname "$0")/../.." || exit 1
O=$(pwd)/gpurun_out
PLAN=shipped,fused_adam,fused_adam_w2 ROUNDS=3 timeout -k 10 500 python scripts/probes/r4_plan_probe.py 300 > $O/r4_31_plans.txt 2>&1 || exit 1
