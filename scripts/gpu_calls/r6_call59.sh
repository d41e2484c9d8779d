#!/bin/bash
# round-6 GPU call 59: qsim12_mfma.hip, qsc_mfma.hip and qsim_mfma.hip also without the SI load/store optimizer
# (lib_b, QDML_NOLSO_FILES; its pairs of 4-byte LDS accesses bank on 32 dwords) against the current library: kernel
# tests on lib_b, then P256 (3 rounds) and P128 (2 rounds) alternating
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_59
mkdir -p $O
L=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd
timeout -k 10 600 env QDML_LIB_DIR=$L/lib_b python -u -m pytest tests/test_kernels_gpu.py tests/test_lds_poison_gpu.py -x -q --timeout 240 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B p256_cur_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12
  B p256_nolso_$r env QDML_LIB_DIR=$L/lib_b python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12
done
for r in 1 2; do
  B p128_nolso_$r env QDML_LIB_DIR=$L/lib_b python bench.py --steps 300 --warmup 20
  B p128_cur_$r python bench.py --steps 300 --warmup 20
done
