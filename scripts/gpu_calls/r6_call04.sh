#!/bin/bash
# round-6 GPU call 4: the library built WITHOUT packed-FP32 instructions (the hazard's fix): full GPU suite (the
# shared-GPU DP test now strict) + smoke, then the benches: the driver's command 2x, 300 steps, fp8, P256/12q,
# BASELINE config 5 (16 qubits + QuantumNAT + gradient pruning + fp8)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -s -k "not test_lds_poison" > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log; grep "pkfma WAR" $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_lds_poison_gpu.py -x -q --timeout 240 --timeout-method thread > $O/${P}_pytest_poison.log 2>&1 || { tail -20 $O/${P}_pytest_poison.log; exit 1; }
tail -1 $O/${P}_pytest_poison.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${P}_smoke.log 2>&1 || { tail -20 $O/${P}_smoke.log; exit 1; }
tail -1 $O/${P}_smoke.log
B() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['value'], d['replays'][:5], d['step_spread']['median_ms'] if d['step_spread'] else None, d['final_losses'])"; }
B bench20 --gpus 1 --steps 20 --warmup 5
B bench20_2 --gpus 1 --steps 20 --warmup 5
B bench --steps 300 --warmup 20
B bench_fp8 --steps 300 --warmup 20 --dtype fp8
B bench_p256 --steps 100 --warmup 10 --pilot 256 --qubits 12
B bench_q16 --steps 20 --warmup 3 --qubits 16 --gradient-pruning --dtype fp8
