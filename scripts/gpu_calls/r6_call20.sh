#!/bin/bash
# round-6 GPU call 20: P256 / 12 qubits in the step -- the conv forward on conv3x3_split_kernel (sps 5: the 32-channel
# layers 23.4 against 27.2 us alone, profiles/r6_18_conv_split_probe_kernel_stats.md) against conv3x3_kernel, 3 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_20
mkdir -p $O
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B base_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12
  B split5_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --knob conv_fwd_split=1 --knob conv_sps=5
done
