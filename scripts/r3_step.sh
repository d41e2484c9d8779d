#!/bin/bash
# Round 3: the fused FC Adam + in-place n<=12 simulator -- tests, then same-box step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu \
  tests/test_flagship_gpu.py::test_fused_fc_adam_matches_separate_adam tests/test_kernels_gpu.py -k "fused or qsim_big" \
  > $OUT/r3_step_tests.log 2>&1 || { tail -30 $OUT/r3_step_tests.log; exit 1; }
tail -2 $OUT/r3_step_tests.log
STEPS=variants VARIANTS="${VARIANTS:-NONE=0|;QDML_FUSED_ADAM=0|;NONE=0|--hdce-branches=w;QDML_FUSED_ADAM=0|--hdce-branches=wa}" bash scripts/gpu_check.sh || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --pilot 256 --qubits 12 > $OUT/p256.log 2>&1 || { tail -20 $OUT/p256.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $OUT/p256.log
