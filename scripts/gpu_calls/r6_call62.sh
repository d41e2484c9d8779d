#!/bin/bash
# round-6 GPU call 62: the final tree (after calls 53-61): full GPU suite + LDS
# poison + smoke; the headline benches (the driver's command twice, --steps 300, no arguments, fp8, P256, P256 x 1024,
# BASELINE config 5, --scaling strong, forced world-1 DP); the default step's kernel stats and timeline
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_62
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "not test_lds_poison" > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_lds_poison_gpu.py -x -q --timeout 240 --timeout-method thread > $O/${P}_pytest_poison.log 2>&1 || { tail -20 $O/${P}_pytest_poison.log; exit 1; }
tail -1 $O/${P}_pytest_poison.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${P}_smoke.log 2>&1 || { tail -20 $O/${P}_smoke.log; exit 1; }
tail -1 $O/${P}_smoke.log
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); s=d.get('step_spread') or {}; print('$n', d['ms_per_step'], d['value'], d['replays'][:4], s.get('median_ms'), d.get('steps_trained'), d['final_losses'])"; }
B bench20 python bench.py --gpus 1 --steps 20 --warmup 5
B bench20_2 python bench.py --gpus 1 --steps 20 --warmup 5
B bench python bench.py --steps 300 --warmup 20
B bench_noargs python bench.py
B bench_fp8 python bench.py --steps 300 --warmup 20 --dtype fp8
B bench_p256 python bench.py --steps 100 --warmup 10 --pilot 256 --qubits 12
B bench_p256_b1024 python bench.py --steps 30 --warmup 5 --pilot 256 --qubits 12 --batch 1024
B bench_q16 python bench.py --steps 30 --warmup 5 --qubits 16 --gradient-pruning --dtype fp8
B bench_strong python bench.py --steps 300 --warmup 20 --scaling strong
B bench_forced env QDML_FORCE_DIST=1 python bench.py --steps 200 --warmup 20
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_prof -o run -- python3 $R/bench.py --steps 200 --warmup 20 > $O/${P}_prof.log 2>&1 || { tail -5 $O/${P}_prof.log; exit 1; }
db=$(find $O/${P}_prof -name '*.db' | head -1)
python scripts/prof_summary.py $db --tail 0.6 > $O/${P}_step_kernel_stats.md 2>&1; head -24 $O/${P}_step_kernel_stats.md
python scripts/prof_timeline.py $db > $O/${P}_step_timeline.md 2>&1; head -5 $O/${P}_step_timeline.md
rm -rf $O/${P}_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_qprof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --qubits 16 --gradient-pruning --dtype fp8 > $O/${P}_qprof.log 2>&1 || { tail -5 $O/${P}_qprof.log; exit 1; }
db=$(find $O/${P}_qprof -name '*.db' | head -1)
python scripts/prof_summary.py $db --tail 0.6 > $O/${P}_q16_kernel_stats.md 2>&1; head -16 $O/${P}_q16_kernel_stats.md
rm -rf $O/${P}_qprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_pprof -o run -- python3 $R/bench.py --steps 60 --warmup 10 --pilot 256 --qubits 12 > $O/${P}_pprof.log 2>&1 || { tail -5 $O/${P}_pprof.log; exit 1; }
db=$(find $O/${P}_pprof -name '*.db' | head -1)
python scripts/prof_summary.py $db --tail 0.6 > $O/${P}_p256_kernel_stats.md 2>&1; head -16 $O/${P}_p256_kernel_stats.md
rm -rf $O/${P}_pprof
