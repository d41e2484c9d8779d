#!/bin/bash
# round-6 GPU call 37: conv layer 1 alone on conv3x3_split_kernel at 12 samples per workgroup (KNOBS.conv_l1_split;
# alone it took 7.6 against 9.1 us in call 18): conv tests, the bench alternating base / l1-split, 3 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_37
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 240 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B base_$r python bench.py --steps 300 --warmup 20
  B l1_$r python bench.py --steps 300 --warmup 20 --knob conv_l1_split=1
done
