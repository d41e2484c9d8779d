#!/bin/bash
# round-6 GPU call 3: the pk_fma WAR probe (uniformity through ds_bpermute), the driver's bench command 3x with the
# replay plan calibrated from a fitted submission cost, one 300-step bench
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_03
timeout -k 10 120 python scripts/probes/probe_pkfma_war.py 2000 256 > $O/${P}_pkfma_war.txt 2>&1 || { tail -20 $O/${P}_pkfma_war.txt; exit 1; }
cat $O/${P}_pkfma_war.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${P}_bench20_$i.json 2>$O/${P}_bench20_$i.err || exit 1
  python -c "import json; d=json.load(open('$O/${P}_bench20_$i.json')); print('bench20', d['ms_per_step'], d['replays'], d['replay_rates_ms'], d['host_ms_per_step'], d['step_spread'])"
done
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/${P}_bench.json 2>$O/${P}_bench.err || exit 1
python -c "import json; d=json.load(open('$O/${P}_bench.json')); print('bench300', d['ms_per_step'], d['replays'][:6], d['replay_rates_ms'], d['step_spread'], d['final_losses'])"
# the DP plan with the independent QSC chain (dp_qsc "indep"): bit-exact against the 5-graph plan over RCCL at world 1,
# then the forced world-1 DP bench with every placement timed (plan_select_ms) and the non-DP step beside it
timeout -k 10 400 python -u -m pytest tests/test_flagship_gpu.py -x -q --timeout 300 --timeout-method thread -k "one_graph" > $O/${P}_pytest_dp.log 2>&1 || { tail -30 $O/${P}_pytest_dp.log; exit 1; }
tail -2 $O/${P}_pytest_dp.log
QDML_FORCE_DIST=1 timeout -k 10 400 python bench.py --steps 200 --warmup 20 > $O/${P}_bench_forced.json 2>$O/${P}_bench_forced.err || { tail -20 $O/${P}_bench_forced.err; exit 1; }
python -c "import json; d=json.load(open('$O/${P}_bench_forced.json')); print('forced', d['ms_per_step'], d['config']['plan_select_ms'], d['config']['dp_qsc'], d['config']['dp_plan'])"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/${P}_bench_nodp.json 2>$O/${P}_bench_nodp.err || exit 1
python -c "import json; d=json.load(open('$O/${P}_bench_nodp.json')); print('non-dp', d['ms_per_step'])"
