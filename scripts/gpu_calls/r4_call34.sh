#!/bin/bash
# round-4 consolidation after the conv VALU diet: full GPU suite, bench, forced-DP bench, P256 / 16-qubit / fp8 benches, step profile
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r4_34_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/r4_34_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r4_34_bench.json 2>$O/r4_34_bench.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --dtype fp8 > $O/r4_34_bench_fp8.json 2>$O/r4_34_bench_fp8.err || exit 1
QDML_FORCE_DIST=1 timeout -k 10 400 python bench.py --steps 200 --warmup 20 --select-steps 30 > $O/r4_34_bench_forced.json 2>$O/r4_34_bench_forced.err || exit 1
timeout -k 10 300 python bench.py --pilot 256 --qubits 12 --steps 100 --warmup 10 > $O/r4_34_bench_p256.json 2>$O/r4_34_bench_p256.err || exit 1
timeout -k 10 300 python bench.py --qubits 16 --dtype fp8 --steps 20 --warmup 3 > $O/r4_34_bench_q16.json 2>$O/r4_34_bench_q16.err || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/prof_step.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_step/run_kernel_trace.csv --tail 0.6 > $O/r4_34_step_kernel_stats.md
python scripts/prof_timeline.py $O/prof_step/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r4_34_step_timeline.md; rm -rf $O/prof_step
