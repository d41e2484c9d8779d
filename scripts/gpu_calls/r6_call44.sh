#!/bin/bash
# round-6 GPU call 44: the fp8 estimator's FC weight gradient in bf16 (KNOBS.f8_wgrad=0: the e4m3 wgrad took 47 against
# the bf16 one's 42 us in the step, profiles/r5_20_*) with the e4m3 data gradient kept: fp8 bench alternating, 3 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_44
mkdir -p $O
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B f8w_$r python bench.py --steps 300 --warmup 20 --dtype fp8
  B bf16w_$r python bench.py --steps 300 --warmup 20 --dtype fp8 --knob f8_wgrad=0
done
B bf16 python bench.py --steps 300 --warmup 20
