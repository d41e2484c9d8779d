#!/bin/bash
# Round-3 GPU call: the 8-qubit circuit forward on the matrix cores (tests + same-box step A/B).  Every GPU
# step has its own limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qsc_gpu.py \
  tests/test_kernels_gpu.py -m gpu > $OUT/pytest_qsc.log 2>&1
rc=$?; tail -3 $OUT/pytest_qsc.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
STEPS="variants" VARIANTS="${VARIANTS:-NONE=0|;QDML_QSIM_MFMA=0|}" bash scripts/gpu_check.sh
