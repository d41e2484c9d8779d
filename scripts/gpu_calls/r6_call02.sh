#!/bin/bash
# round-6 GPU call 2: the pk_fma WAR probe with a lane dump, the conv stack alone with / without the pipelined
# kernels, and the driver's bench command 3x with the calibrated replay plan
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_02
timeout -k 10 120 python scripts/probes/probe_pkfma_war.py 2000 256 > $O/${P}_pkfma_war.txt 2>&1 || { tail -20 $O/${P}_pkfma_war.txt; exit 1; }
cat $O/${P}_pkfma_war.txt
timeout -k 10 200 python scripts/probes/probe_conv_db.py 40 > $O/${P}_conv_db.txt 2>&1 || { tail -20 $O/${P}_conv_db.txt; exit 1; }
cat $O/${P}_conv_db.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${P}_bench20_$i.json 2>$O/${P}_bench20_$i.err || exit 1
  python -c "import json; d=json.load(open('$O/${P}_bench20_$i.json')); print('bench20', d['ms_per_step'], d['replays'], d['replay_rates_ms'], d['host_ms_per_step'], d['step_spread'])"
done
