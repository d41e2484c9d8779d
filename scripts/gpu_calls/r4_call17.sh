#!/bin/bash
# round-4 GPU call: conv forward prefetch rework -- conv numerics + LDS-poison + bit-exact plans, phase stamps, bench +
# step timeline
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_lds_poison_gpu.py tests/test_flagship_gpu.py -q --timeout 200 --timeout-method thread > $O/r4_17_pytest.log 2>&1; echo "pytest rc=$?" >> $O/r4_17_pytest.log
timeout -k 10 120 python scripts/probes/stamp_conv.py > $O/r4_17_stamp_conv.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r4_17_bench.json 2>$O/r4_17_bench.err || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/tl_step.log 2>&1) || exit 1
python scripts/prof_timeline.py $O/tl_step/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r4_17_step_timeline.md
python scripts/prof_summary.py $O/tl_step/run_kernel_trace.csv --tail 0.6 > $O/r4_17_step_kernel_stats.md; rm -rf $O/tl_step
