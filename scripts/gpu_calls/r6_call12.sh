#!/bin/bash
# round-6 GPU call 12: graph executables destroyed only at exit (QDML_GRAPH_RELEASE=exit) after call 11's second
# host segfault (profiles/r6_11b_bench_forced_segfault.txt): full GPU suite + smoke; the forced world-1 DP bench
# (plan selection: candidates closed) twice; the default step's kernel stats and timeline
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_12
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${P}_smoke.log 2>&1 || { tail -20 $O/${P}_smoke.log; exit 1; }
tail -1 $O/${P}_smoke.log
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -45 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); s=d.get('step_spread') or {}; print('$n', d['ms_per_step'], d['value'], d['replays'][:4], s.get('median_ms'), d.get('steps_trained'), d['config'].get('plan_select_ms'), d['final_losses'])"; }
B bench_forced env QDML_FORCE_DIST=1 python bench.py --steps 200 --warmup 20
B bench_forced_2 env QDML_FORCE_DIST=1 python bench.py --steps 200 --warmup 20
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_prof -o run -- python3 $R/bench.py --steps 200 --warmup 20 > $O/${P}_prof.log 2>&1 || { tail -5 $O/${P}_prof.log; exit 1; }
db=$(find $O/${P}_prof -name '*.db' | head -1)
python scripts/prof_summary.py $db --tail 0.6 > $O/${P}_step_kernel_stats.md 2>&1; head -24 $O/${P}_step_kernel_stats.md
python scripts/prof_timeline.py $db > $O/${P}_step_timeline.md 2>&1; head -5 $O/${P}_step_timeline.md
rm -rf $O/${P}_prof
