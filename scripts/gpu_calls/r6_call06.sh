#!/bin/bash
# round-6 GPU call 6: QSC chain workgroup counts that give every wave the same number of samples (2304 samples,
# 4 waves per workgroup: 256 workgroups = 2.25 samples per wave, so a quarter of the waves run a third sample while
# the rest wait at the slab reduction's barrier; 192 = 3 each, 144 = 4 each), forward cap and backward grid, against
# the default, alternating, 3 rounds, --steps 300; then bf16 vs fp8 alternating, 3 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_06
B() { n=$1; shift; timeout -k 10 300 python bench.py --steps 300 --warmup 20 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['replay_rates_ms']['gpu'], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses']['qsc_nll'], d['final_losses']['hdce_nmse'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B def_$r
  B f192b192_$r --knob qsc_fwd_cap=192 --qsc-grid-bwd 192
  B f144b144_$r --knob qsc_fwd_cap=144 --qsc-grid-bwd 144
  B b192_$r --qsc-grid-bwd 192
  B f192_$r --knob qsc_fwd_cap=192
done
for r in 1 2 3; do
  B bf16_$r
  B fp8_$r --dtype fp8
done
