#!/bin/bash
# round-6 GPU call 42: P256's QSC preprocess backward grid (qsc2_bwd_kernel<16,16,2>: tuned at P128; the balanced cap
# gives 231 two-wave workgroups of 5 samples per wave): --qsc-grid-bwd 0 (default) / 384 / 576 / 1152, 2 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_42
mkdir -p $O
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2; do
  for g in 0 384 576 1152; do
    B g${g}_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --qsc-grid-bwd $g
  done
done
