#!/bin/bash
# round-5 final consolidation: full GPU suite + smoke on the final round-5 tree, the headline benches and the
# default step's kernel stats + timeline (plus a second and third default bench: the QSC loss run to run)

set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5_46_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/r5_46_pytest.log
tail -3 $O/r5_46_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r5_46_smoke.log 2>&1 || { tail -20 $O/r5_46_smoke.log; exit 1; }
tail -2 $O/r5_46_smoke.log
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r5_46_bench.json 2>$O/r5_46_bench.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r5_46_bench_2.json 2>$O/r5_46_bench_2.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r5_46_bench_3.json 2>$O/r5_46_bench_3.err || exit 1
timeout -k 10 120 python bench.py > $O/r5_46_bench_default_args.json 2>$O/r5_46_bench_default_args.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --dtype fp8 > $O/r5_46_bench_fp8.json 2>$O/r5_46_bench_fp8.err || exit 1
QDML_FORCE_DIST=1 timeout -k 10 400 python bench.py --steps 200 --warmup 20 --select-steps 30 > $O/r5_46_bench_forced.json 2>$O/r5_46_bench_forced.err || exit 1
timeout -k 10 300 python bench.py --pilot 256 --qubits 12 --steps 100 --warmup 10 > $O/r5_46_bench_p256.json 2>$O/r5_46_bench_p256.err || exit 1
timeout -k 10 300 python bench.py --pilot 256 --qubits 12 --batch 1024 --steps 30 --warmup 5 > $O/r5_46_bench_p256_b1024.json 2>$O/r5_46_bench_p256_b1024.err || exit 1
timeout -k 10 300 python bench.py --qubits 16 --dtype fp8 --steps 20 --warmup 3 > $O/r5_46_bench_q16.json 2>$O/r5_46_bench_q16.err || exit 1
cat $O/r5_46_bench.json $O/r5_46_bench_fp8.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/prof_step.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_step/run_kernel_trace.csv --tail 0.6 > $O/r5_46_step_kernel_stats.md
python scripts/prof_timeline.py $O/prof_step/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r5_46_step_timeline.md; rm -rf $O/prof_step
head -40 $O/r5_46_step_timeline.md
