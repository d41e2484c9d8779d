#!/bin/bash
# round-6 GPU call 43: P256's other conv launch shapes (tuned at P128): forward samples per wave (conv_spw 2 / 3 / 4)
# and layer 1's weight-gradient samples per workgroup (conv_spb_w1 2 / 4 / 8), 2 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_43
mkdir -p $O
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2; do
  B base_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12
  B spw2_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --knob conv_spw=2
  B spw4_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --knob conv_spw=4
  B w1_2_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --knob conv_spb_w1=2
  B w1_8_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --knob conv_spb_w1=8
done
