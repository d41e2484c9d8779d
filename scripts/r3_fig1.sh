#!/bin/bash
# Round 3: FIG1 with the HDCE trained in bf16 on the fused HIP step (the shipped path) and in fp32 through the
# torch autograd step (hdce_engine=torch, dtype fp32, evaluated in fp32 too) -- the 15 dB attribution.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python scripts/train_eval.py --epochs ${EPOCHS:-100} --qubits 6 --out $OUT/r3_fig1_bf16 \
  --workspace /tmp/ws_bf16 > $OUT/r3_fig1_bf16.log 2>&1 || { tail -30 $OUT/r3_fig1_bf16.log; exit 1; }
tail -2 $OUT/r3_fig1_bf16.log
QDML_EVAL_TORCH=1 timeout -k 10 900 python scripts/train_eval.py --epochs ${EPOCHS:-100} --qubits 6 --dtype fp32 \
  --hdce-engine torch --out $OUT/r3_fig1_fp32 --workspace /tmp/ws_fp32 > $OUT/r3_fig1_fp32.log 2>&1 || { tail -30 $OUT/r3_fig1_fp32.log; exit 1; }
tail -2 $OUT/r3_fig1_fp32.log
