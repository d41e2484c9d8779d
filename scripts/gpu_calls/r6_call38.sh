#!/bin/bash
# round-6 GPU call 38: P256's fused conv backward runs one workgroup per CU (131 KB of LDS at W = 16), so spb 5's 468
# workgroups make two rounds; spb 8 (288) / 10 (234) against the default 5 in the P256 step, 2 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_38
mkdir -p $O
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2; do
  B spb5_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12
  B spb8_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --knob conv_spb_f=8
  B spb10_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --knob conv_spb_f=10
done
