#!/bin/bash
# round-6 GPU call 61: the one-tile reverse pass A storing lambda from its second LDS group straight to HBM (QD_STREAM_A1T_OUT2:
# the register bits undone first, no tile write-back + read-back) against QD_STREAM_A1T_OUT2=0 (lib_base): kernel tests
# + LDS poison, the probe and config 5 alternating, 2 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_61
mkdir -p $O
L=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_lds_poison_gpu.py -x -q --timeout 240 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u scripts/probes/probe_qstream.py 6 2>&1 | grep n=16 | sed "s/^/new  /" | tee -a $O/${P}_probe.txt || exit 1
  timeout -k 10 200 env QDML_LIB_DIR=$L/lib_base python -u scripts/probes/probe_qstream.py 6 2>&1 | grep n=16 | sed "s/^/base /" | tee -a $O/${P}_probe.txt || exit 1
done
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2; do
  B new_$r python bench.py --steps 30 --warmup 5 --qubits 16 --gradient-pruning --dtype fp8
  B base_$r env QDML_LIB_DIR=$L/lib_base python bench.py --steps 30 --warmup 5 --qubits 16 --gradient-pruning --dtype fp8
done
