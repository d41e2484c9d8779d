#!/bin/bash
# round-5 GPU call 22: timeline of the fp8 step with layer 3's BN backward reduction in the e4m3 data gradient's
# epilogue (r5_21: no step gain -- where did the 20 us of bn_bwd_reduce go?)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f8b -o run -- python $R/bench.py --steps 100 --warmup 20 --dtype fp8 > $O/prof_f8b.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_f8b/run_kernel_trace.csv --tail 0.6 > $O/r5_22_fp8_bnred_kernel_stats.md
python scripts/prof_timeline.py $O/prof_f8b/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r5_22_fp8_bnred_timeline.md; rm -rf $O/prof_f8b
head -34 $O/r5_22_fp8_bnred_timeline.md
