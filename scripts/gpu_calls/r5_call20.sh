#!/bin/bash
# round-5 GPU call 20: kernel stats + timeline of the fp8-estimator step (why it is only ~1 % faster than bf16 when its
# e4m3 FC GEMMs are 25-40 % faster alone), and of the bf16 step on the same box for comparison
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
for v in fp8 bf16; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python $R/bench.py --steps 100 --warmup 20 --dtype $v > $O/prof_$v.log 2>&1) || exit 1
  python scripts/prof_summary.py $O/prof_$v/run_kernel_trace.csv --tail 0.6 > $O/r5_20_${v}_kernel_stats.md
  python scripts/prof_timeline.py $O/prof_$v/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r5_20_${v}_timeline.md; rm -rf $O/prof_$v
done
head -40 $O/r5_20_fp8_timeline.md
