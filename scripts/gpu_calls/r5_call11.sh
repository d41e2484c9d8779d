#!/bin/bash
# round-5 GPU call 11: (1) conv GPU tests incl. the persistent forward (conv_fwd_stack_kernel) against the per-layer
# launches; (2) step A/B: conv.hip before the prologue change (commit 553c2ae, lib/libqdml_hip_base.so swapped in,
# scripts/build_ab_lib.sh) / the current library / + the persistent forward (--knob conv_stack=1), 3 alternating
# rounds; (3) the indep plan's bit-exact test with 8 trials; (4) FIG1 with the HDCE weight average + test-time BN
# adaptation, K = 10 and 30 (reference protocol otherwise); (5) P256 dagq vs indep
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; L=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r5_11_pytest.log 2>&1 || { tail -40 $O/r5_11_pytest.log; exit 1; }
tail -1 $O/r5_11_pytest.log
cp $L/libqdml_hip.so /tmp/new.so
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_11_cur.json 2> $O/r5_11_cur.err || { tail -20 $O/r5_11_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_11_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_11_ab.txt
}
for r in 1 2 3; do
  cp $L/libqdml_hip_base.so $L/libqdml_hip.so; run "r$r base"
  cp /tmp/new.so $L/libqdml_hip.so; run "r$r prologue"
  run "r$r stack" --knob conv_stack=1
done
QDML_BITEXACT_TRIALS=8 timeout -k 10 300 python -u -m pytest tests/test_flagship_gpu.py -x -q -k "bit_exact and indep" --timeout 280 --timeout-method thread > $O/r5_11_bitexact.log 2>&1 || { tail -30 $O/r5_11_bitexact.log; exit 1; }
tail -1 $O/r5_11_bitexact.log
for K in 10 30; do
  timeout -k 10 900 python -u scripts/train_eval.py --epochs 100 --qubits 6 --out $O/r5_fig1_swa$K --workspace /tmp/ws_swa$K \
    --bn-adapt --swa-epochs $K > $O/r5_11_fig1_swa$K.log 2>&1 || { tail -30 $O/r5_11_fig1_swa$K.log; exit 1; }
  tail -1 $O/r5_11_fig1_swa$K.log
done
for r in 1 2; do
  for v in dagq indep; do
    timeout -k 10 200 python bench.py --pilot 256 --qubits 12 --steps 100 --warmup 10 --stream-mode $v > $O/r5_11_cur.json 2> $O/r5_11_cur.err || { tail -20 $O/r5_11_cur.err; exit 1; }
    echo "round $r [p256 $v] $(python -c "import json; d=json.load(open('$O/r5_11_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'])")" | tee -a $O/r5_11_p256_ab.txt
  done
done
