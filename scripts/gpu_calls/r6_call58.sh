#!/bin/bash
# round-6 GPU call 58: (call 57 with the order reversed: base first) the P128 step on the current library (qsim_stream.hip changes of calls 53-55 and a full rebuild)
# against the call-52 tree's library (lib_base, built from 66bbcdf) -- P128 does not run qsim_stream.hip, so the two
# should be level -- --steps 300, alternating, 3 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_58
mkdir -p $O
L=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B base_$r env QDML_LIB_DIR=$L/lib_base python bench.py --steps 300 --warmup 20
  B new_$r python bench.py --steps 300 --warmup 20
done
