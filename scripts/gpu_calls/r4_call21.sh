#!/bin/bash
# round-4 GPU call: the HDCE loss in the FC forward's epilogue (hand "fwd") on the 4-stage tile vs the shipped plain
# forward + one-pass NMSE, 3 rounds; GEMM NMSE-epilogue numerics first
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 120 --timeout-method thread -k "nmse" > $O/r4_21_pytest.log 2>&1; echo "pytest rc=$?" >> $O/r4_21_pytest.log
ROUNDS=3 PLAN=shipped,fused_loss6 timeout -k 10 500 python scripts/probes/r4_plan_probe.py 400 > $O/r4_21_plans.txt 2>&1 || exit 1
