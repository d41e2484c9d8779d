#!/bin/bash
# Round 3: FIG1 with the fp8 estimator (e4m3 FC forward + weight / data gradients on the MX-scaled MFMA, bf16
# convs) vs the bf16 one, same box, same protocol; then the fp8 GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python scripts/train_eval.py --epochs ${EPOCHS:-100} --qubits 6 --out $OUT/r3_fig1_bf16b \
  --workspace /tmp/ws_bf16 > $OUT/r3_fig1_bf16b.log 2>&1 || { tail -30 $OUT/r3_fig1_bf16b.log; exit 1; }
tail -2 $OUT/r3_fig1_bf16b.log
timeout -k 10 600 python scripts/train_eval.py --epochs ${EPOCHS:-100} --qubits 6 --dtype fp8 --out $OUT/r3_fig1_fp8 \
  --workspace /tmp/ws_fp8 > $OUT/r3_fig1_fp8.log 2>&1 || { tail -30 $OUT/r3_fig1_fp8.log; exit 1; }
tail -2 $OUT/r3_fig1_fp8.log
