#!/bin/bash
# round-6 GPU call 5: the cost of building without packed-FP32 instructions, on one box: bench 300 steps alternating
# the shipped library (lib/) and the packed build (lib_pk/, QDML_PACKED_F32=1), 3 rounds; then a kernel-trace profile
# of each (per-kernel time: which kernels lost)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_05
PK=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd/lib_pk
B() { n=$1; shift; timeout -k 10 300 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:5], d['replay_rates_ms'], d['step_spread']['median_ms'], d['final_losses']['qsc_nll'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B nopk_$r python bench.py --steps 300 --warmup 20
  B pk_$r env QDML_LIB_DIR=$PK python bench.py --steps 300 --warmup 20
done
for v in nopk pk; do
  if [ $v = pk ]; then export QDML_LIB_DIR=$PK; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_prof_$v -o run -- python3 $R/bench.py --steps 200 --warmup 20 > $O/${P}_prof_$v.log 2>&1 || { tail -5 $O/${P}_prof_$v.log; exit 1; }
  db=$(find $O/${P}_prof_$v -name '*.db' | head -1)
  python scripts/prof_summary.py $db --tail 0.6 > $O/${P}_kernel_stats_$v.md 2>&1
  head -40 $O/${P}_kernel_stats_$v.md
done
