#!/bin/bash
# round-6 GPU call 14: kernel stats of the P256 / 12-qubit step (what its 1.1 ms is made of on the round-6 tree)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_14
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_prof -o run -- python3 $R/bench.py --steps 60 --warmup 10 --pilot 256 --qubits 12 > $O/${P}_prof.log 2>&1 || { tail -5 $O/${P}_prof.log; exit 1; }
db=$(find $O/${P}_prof -name '*.db' | head -1)
python scripts/prof_summary.py $db --tail 0.6 > $O/${P}_p256_kernel_stats.md 2>&1; head -40 $O/${P}_p256_kernel_stats.md
rm -rf $O/${P}_prof
