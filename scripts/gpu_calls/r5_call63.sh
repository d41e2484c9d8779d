#!/bin/bash
# round-5 GPU call 63: the final tree (conv1 weights through readfirstlane, k loop unrolled 3): full GPU suite + smoke, the default
# bench twice and the fp8 bench
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5_63_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/r5_63_pytest.log
tail -3 $O/r5_63_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r5_63_smoke.log 2>&1 || { tail -20 $O/r5_63_smoke.log; exit 1; }
tail -1 $O/r5_63_smoke.log
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r5_63_bench.json 2>$O/r5_63_bench.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r5_63_bench_2.json 2>$O/r5_63_bench_2.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --dtype fp8 > $O/r5_63_bench_fp8.json 2>$O/r5_63_bench_fp8.err || exit 1
for f in bench bench_2 bench_fp8; do python -c "import json; d=json.load(open('$O/r5_63_$f.json')); print('$f', d['ms_per_step'], d['value'], d['final_losses'])"; done
