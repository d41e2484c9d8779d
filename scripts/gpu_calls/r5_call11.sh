#!/bin/bash
# round-5 GPU call 11: FIG1 with the HDCE weight average (RunnerConfig.swa_epochs) and test-time BN adaptation,
# the reference protocol otherwise (100 epochs, training SNR 10 dB, 10k test samples per SNR); K = 10 and 30
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
O=$(pwd)/gpurun_out
for K in 10 30; do
  timeout -k 10 900 python -u scripts/train_eval.py --epochs 100 --qubits 6 --out $O/r5_fig1_swa$K --workspace /tmp/ws_swa$K \
    --bn-adapt --swa-epochs $K > $O/r5_11_fig1_swa$K.log 2>&1 || { tail -30 $O/r5_11_fig1_swa$K.log; exit 1; }
  tail -1 $O/r5_11_fig1_swa$K.log
done
