#!/bin/bash
# conv backward staging in packed pairs (dz = c1 g - (k3 z + k0)): conv tests, A/B vs the previous library, timeline
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r4_30_pytest.log 2>&1 || exit 1
bash scripts/ab_lib.sh r4_30 3 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/prof_step.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_step/run_kernel_trace.csv --tail 0.6 > $O/r4_30_step_kernel_stats.md
python scripts/prof_timeline.py $O/prof_step/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r4_30_step_timeline.md; rm -rf $O/prof_step
