#!/bin/bash
# round-6 GPU call 15: P256's QSC forward with conv1 on f32 MFMAs (conv1_mfma16: 186 VGPRs, 2 waves per SIMD instead of
# 1) -- QSC tests incl. the pool-1 map / choices against torch at P128 and P256; the P256 bench alternating new / base
# (lib_base = HEAD before this change) / new + the bf16x3 conv2 forward (KNOBS.qsc_fwd3_p256), 3 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_15
BASE=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd/lib_base
timeout -k 10 600 python -u -m pytest tests/test_qsc_gpu.py -x -q -s --timeout 240 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log; grep "pool-1 vs torch\|conv1 MFMA" $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B new_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12
  B base_$r env QDML_LIB_DIR=$BASE python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12
  B fwd3_$r python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12 --knob qsc_fwd3_p256=1
done
