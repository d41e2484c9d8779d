#!/bin/bash
# round-6 GPU call 1: the round's first tree (graph lifetime in the product code, no conftest teardown, crash
# handler, [1, 4, 15] replay plan, strong-scaling / pruning flags; the pipelined conv forward A/B): full GPU suite + smoke, the driver's bench
# command twice, a 300-step bench, and a kernel-stats profile of the default step
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_01
timeout -k 10 120 python scripts/probes/probe_pkfma_war.py 4000 256 > $O/${P}_pkfma_war.txt 2>&1 || { tail -20 $O/${P}_pkfma_war.txt; exit 1; }
cat $O/${P}_pkfma_war.txt
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k pipelined > $O/${P}_pytest_db.log 2>&1 || { tail -30 $O/${P}_pytest_db.log; exit 1; }
tail -2 $O/${P}_pytest_db.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${P}_smoke.log 2>&1 || { tail -20 $O/${P}_smoke.log; exit 1; }
tail -1 $O/${P}_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${P}_bench20.json 2>$O/${P}_bench20.err || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${P}_bench20_2.json 2>$O/${P}_bench20_2.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/${P}_bench.json 2>$O/${P}_bench.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --knob conv_fwd_db=1 > $O/${P}_bench_db.json 2>$O/${P}_bench_db.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/${P}_bench_2.json 2>$O/${P}_bench_2.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --knob conv_fwd_db=1 > $O/${P}_bench_db_2.json 2>$O/${P}_bench_db_2.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --knob conv_fwd_db=1 --knob conv_bwd_db=1 > $O/${P}_bench_db2.json 2>$O/${P}_bench_db2.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --knob conv_fwd_db=1 --knob conv_bwd_db=1 > $O/${P}_bench_db2_2.json 2>$O/${P}_bench_db2_2.err || exit 1
for f in bench20 bench20_2 bench bench_db bench_2 bench_db_2 bench_db2 bench_db2_2; do python -c "import json; d=json.load(open('$O/${P}_$f.json')); print('$f', d['ms_per_step'], d['replays'][:5], d['step_spread'], d['final_losses'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_prof -o run -- python3 $R/bench.py --steps 200 --warmup 20 --knob conv_fwd_db=1 --knob conv_bwd_db=1 > $O/${P}_prof.log 2>&1 || exit 1
cd $R && python scripts/prof_summary.py $(ls $O/${P}_prof/*/run_kernel_trace.csv $O/${P}_prof/run_kernel_trace.csv 2>/dev/null | head -1) --tail 0.6 > $O/${P}_kernel_stats.md 2>&1; head -30 $O/${P}_kernel_stats.md
