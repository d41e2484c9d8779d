#!/bin/bash
# round-4 GPU call: QSC fork placement inside the step (node-creation order vs the executor's queue mapping)
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
PLAN=shipped,fork_conv1,fork_conv2 timeout -k 10 400 python scripts/probes/r4_plan_probe.py 300 > $O/r4_15_plans.txt 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && PLAN=fork_conv1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl_fc1 -o run -- python $R/scripts/probes/r4_plan_probe.py 100 > $O/tl_fc1.log 2>&1) || exit 1
python scripts/prof_timeline.py $O/tl_fc1/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r4_15_timeline_fork_conv1.md; rm -rf $O/tl_fc1
