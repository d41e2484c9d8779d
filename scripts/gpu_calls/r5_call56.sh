#!/bin/bash
# round-5 GPU call 56: conv1's weights made wave-uniform (readfirstlane of the LDS broadcast reads) in the QSC
# preprocess forward: do the graph plans' p1s differences (channel 5, windows 24-31 = lanes 48-63: r5_55) go away;
# the QSC GPU tests and the multistream tests; the default bench and the step's kernel stats
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
for m in fcnext conv; do PROBE_RECOMPUTE=1 timeout -k 10 200 python -u scripts/probes/probe_split_fused.py wgrad $m 1 >> $O/r5_56_uniform_probe.txt 2>&1 || { tail -20 $O/r5_56_uniform_probe.txt; exit 1; }; done
grep "differ\|recompute\|^step\|sample" $O/r5_56_uniform_probe.txt; true
timeout -k 10 600 python -u -m pytest tests/test_qsc_gpu.py tests -k "qsc or multistream" -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5_56_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/r5_56_pytest.log
tail -3 $O/r5_56_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r5_56_bench.json 2>$O/r5_56_bench.err || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r5_56_bench_2.json 2>$O/r5_56_bench_2.err || exit 1
cat $O/r5_56_bench.json $O/r5_56_bench_2.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/prof_step.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_step/run_kernel_trace.csv --tail 0.6 > $O/r5_56_step_kernel_stats.md; rm -rf $O/prof_step
grep "qsc2_fwd\|wall" $O/r5_56_step_kernel_stats.md
