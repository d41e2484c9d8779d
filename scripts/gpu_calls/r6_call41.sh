#!/bin/bash
# round-6 GPU call 41: P256 with the fused conv backward at spb 10 by default (KNOBS.conv_spb_f_w16): conv + flagship
# tests; P256 x 1024 (BASELINE config 4) alternating spb 10 (default) / 5, 2 rounds; the P256 default once
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_41
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_conv_gpu.py tests/test_flagship_gpu.py -x -q --timeout 240 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2; do
  B b1024_spb10_$r python bench.py --steps 30 --warmup 5 --pilot 256 --qubits 12 --batch 1024
  B b1024_spb5_$r python bench.py --steps 30 --warmup 5 --pilot 256 --qubits 12 --batch 1024 --knob conv_spb_f_w16=5
done
B p256 python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12
