#!/bin/bash
# round-6 GPU call 45: the QSC chain's placement re-tested on the round-6 kernels: --qsc-start conv (each step's QSC
# chain waits for the HDCE conv forward, which then has the chip to itself) against the default, 3 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_45
mkdir -p $O
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B base_$r python bench.py --steps 300 --warmup 20
  B conv_$r python bench.py --steps 300 --warmup 20 --qsc-start conv
done
