#!/bin/bash
# round-6 GPU call 34: the last forward pass B forming <Z_q> straight from its registers (5 signed sums of |a|^2: bit q
# of the ring image is a prefix parity) instead of the ring scatter through LDS: kernel tests + LDS poison, the probe,
# config 5 twice
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_34
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_lds_poison_gpu.py -x -q --timeout 240 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u scripts/probes/probe_qstream.py 6 2>&1 | grep n=16 | tee -a $O/${P}_probe.txt
done
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
B q16_1 python bench.py --steps 30 --warmup 5 --qubits 16 --gradient-pruning --dtype fp8
B q16_2 python bench.py --steps 30 --warmup 5 --qubits 16 --gradient-pruning --dtype fp8
