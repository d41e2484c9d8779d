#!/bin/bash
# round-6 GPU call 40: P256's fused conv backward at spb 10 (one round of 234 workgroups) against the default 5 (468:
# two rounds at one workgroup per CU), alternating on one box, 3 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_40
mkdir -p $O
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B spb5_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12
  B spb10_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --knob conv_spb_f=10
done
