#!/bin/bash
# Round 3: the e4m3 FC forward on the MX-scaled MFMA -- numerics, isolated timing, fp8 vs bf16 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -m gpu > $OUT/r3_fp8_tests.log 2>&1 || { tail -30 $OUT/r3_fp8_tests.log; exit 1; }
tail -2 $OUT/r3_fp8_tests.log
timeout -k 10 300 python scripts/probe_gemm.py > $OUT/r3_probe_gemm_f8.log 2>&1 || { tail -20 $OUT/r3_probe_gemm_f8.log; exit 1; }
cat $OUT/r3_probe_gemm_f8.log
STEPS=variants BENCH_STEPS=300 VARIANTS="${VARIANTS:-NONE=0|;NONE=0|--dtype=fp8;QDML_FP8_CONV=0|--dtype=fp8;QDML_F8_MX=0|--dtype=fp8}" bash scripts/gpu_check.sh || exit 1
