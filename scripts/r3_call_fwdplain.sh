#!/bin/bash
# Round-3 GPU call: the hand-written FC forward with a bias-only epilogue + the separate one-pass NMSE kernel
# (QDML_HAND_GEMM=fwdplain) -- test, then same-box step A/B at P128 and P256.  Any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -m gpu \
  -k "plain or fwd_matches" > $OUT/pytest_fwdplain.log 2>&1
rc=$?; tail -3 $OUT/pytest_fwdplain.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
STEPS="variants" VARIANTS="NONE=0|;QDML_HAND_GEMM=fwdplain,wgrad,dgrad QDML_GEMM_CFG=2,1,2|;QDML_HAND_GEMM=fwdplain,wgrad,dgrad QDML_GEMM_CFG=0,1,2|;NONE=0|--pilot 256 --qubits 12;QDML_HAND_GEMM=fwdplain,wgrad,dgrad QDML_GEMM_CFG=2,1,2|--pilot 256 --qubits 12" bash scripts/gpu_check.sh
