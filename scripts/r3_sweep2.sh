#!/bin/bash
# Round 3: HDCE side-branch variants on the new default, the P256 / 12-qubit kernel profile, the 16-qubit step.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
STEPS=variants VARIANTS="${VARIANTS:-NONE=0|;NONE=0|--hdce-branches=w;NONE=0|--hdce-branches=c;NONE=0|--hdce-branches=wc;QDML_FUSED_ADAM=1|--hdce-branches=wc}" bash scripts/gpu_check.sh || exit 1
STEPS=prof_cfg PROF_NAME=p256 PROF_ARGS="--steps 30 --warmup 5 --pilot 256 --qubits 12 --steps-per-graph 1" bash scripts/gpu_check.sh > /dev/null || exit 1
rm -rf $OUT/prof_p256
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --qubits 16 --dtype fp8 > $OUT/q16.log 2>&1 || { tail -20 $OUT/q16.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $OUT/q16.log
head -14 $OUT/prof_p256_summary.md
