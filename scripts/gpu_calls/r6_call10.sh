#!/bin/bash
# round-6 GPU call 10: conv1_mfma with every band's loads in flight, the window rows exchanged by v_permlane32_swap and
# the codes built from two ballots (call 9's form was 2.4k cycles slower than the VALU loop): QSC tests, forward
# stamps new vs base, bench A/B 3 rounds; then the world-1 DP step's kernel trace (forced RCCL, all-reduce / fwd)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_10
BASE=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd/lib_base
timeout -k 10 600 python -u -m pytest tests/test_qsc_gpu.py -x -q -s --timeout 240 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log; grep "conv1 MFMA" $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
for v in new base; do
  if [ $v = base ]; then export QDML_LIB_DIR=$BASE; fi
  timeout -k 10 120 python scripts/probes/stamp_qsc.py > $O/${P}_stamp_fwd_$v.json 2>$O/${P}_stamp_fwd_$v.err || { tail -5 $O/${P}_stamp_fwd_$v.err; exit 1; }
  python -c "import json; a=json.load(open('$O/${P}_stamp_fwd_$v.json')); print('$v fwd', {k: v['median_cycles'] for k, v in a.items() if isinstance(v, dict) and 'median_cycles' in v}, a['wave_lifetime_median_cycles'])"
done
unset QDML_LIB_DIR
B() { n=$1; shift; timeout -k 10 300 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['replay_rates_ms']['gpu'], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses']['qsc_nll'], d['final_losses']['hdce_nmse'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2 3; do
  B new_$r python bench.py --steps 300 --warmup 20
  B base_$r env QDML_LIB_DIR=$BASE python bench.py --steps 300 --warmup 20
done
export QDML_FORCE_DIST=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_prof_dp -o run -- python3 $R/bench.py --steps 200 --warmup 20 --dp-plan allreduce --dp-qsc fwd > $O/${P}_prof_dp.log 2>&1 || { tail -5 $O/${P}_prof_dp.log; exit 1; }
db=$(find $O/${P}_prof_dp -name '*.db' | head -1)
python scripts/prof_summary.py $db --tail 0.6 > $O/${P}_dp_kernel_stats.md 2>&1; head -40 $O/${P}_dp_kernel_stats.md
rm -rf $O/${P}_prof_dp
