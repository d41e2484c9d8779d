#!/bin/bash
# round-5 GPU call 14: the benches call 13 did not reach (P256 x 1024 -- steps per replay now clamped to what a
# stream's permutation holds --, 16 qubits + fp8), the default step's kernel stats + timeline, and the persistent
# conv forward's per-phase stamps (why it is 105 us against 58 for the per-layer launches)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python bench.py --pilot 256 --qubits 12 --batch 1024 --steps 30 --warmup 5 > $O/r5_14_bench_p256_b1024.json 2>$O/r5_14_bench_p256_b1024.err || { tail -5 $O/r5_14_bench_p256_b1024.err; exit 1; }
cat $O/r5_14_bench_p256_b1024.json
timeout -k 10 300 python bench.py --qubits 16 --dtype fp8 --steps 20 --warmup 3 > $O/r5_14_bench_q16.json 2>$O/r5_14_bench_q16.err || { tail -5 $O/r5_14_bench_q16.err; exit 1; }
cat $O/r5_14_bench_q16.json
QDML_STACK_STAMPS=1 timeout -k 10 120 python scripts/probes/probe_conv_stack.py > $O/r5_14_stack_stamps.txt 2>&1 || { cat $O/r5_14_stack_stamps.txt; exit 1; }
cat $O/r5_14_stack_stamps.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/prof_step.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_step/run_kernel_trace.csv --tail 0.6 > $O/r5_14_step_kernel_stats.md
python scripts/prof_timeline.py $O/prof_step/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r5_14_step_timeline.md; rm -rf $O/prof_step
head -45 $O/r5_14_step_timeline.md
