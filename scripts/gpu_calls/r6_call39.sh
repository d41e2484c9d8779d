#!/bin/bash
# round-6 GPU call 39: P256's fused conv backward samples per workgroup around call 38's winner (10: 234 workgroups,
# one round at one per CU): 10 / 11 (216) / 12 (198) / 13 (180), 2 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_39
mkdir -p $O
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2; do
  for b in 10 11 12 13; do
    B spb${b}_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --knob conv_spb_f=$b
  done
done
