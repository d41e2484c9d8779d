#!/bin/bash
# round-6 GPU call 63: the fp8 estimator's step -- kernel stats (--dtype fp8, 200 steps) next to the bf16 step's
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_63
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_prof -o run -- python3 $R/bench.py --steps 200 --warmup 20 --dtype fp8 > $O/${P}_prof.log 2>&1 || { tail -5 $O/${P}_prof.log; exit 1; }
db=$(find $O/${P}_prof -name '*.db' | head -1)
python scripts/prof_summary.py $db --tail 0.6 > $O/${P}_fp8_kernel_stats.md 2>&1; head -30 $O/${P}_fp8_kernel_stats.md
rm -rf $O/${P}_prof
