#!/bin/bash
# round-5 GPU call 16: kernel stats + timeline of the 16-qubit + fp8 step (BASELINE config 5), to size an MFMA pass A
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_q16 -o run -- python $R/bench.py --qubits 16 --dtype fp8 --steps 12 --warmup 3 > $O/prof_q16.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_q16/run_kernel_trace.csv --tail 0.6 > $O/r5_16_q16_kernel_stats.md
python scripts/prof_timeline.py $O/prof_q16/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 3 > $O/r5_16_q16_timeline.md; rm -rf $O/prof_q16
head -30 $O/r5_16_q16_kernel_stats.md
