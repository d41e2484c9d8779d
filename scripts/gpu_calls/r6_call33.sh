#!/bin/bash
# round-6 GPU call 33: the streamed simulator's reverse pass A at 1 / 2 / 4 bricks per workgroup (QDML_QSTREAM_BPB)
# after calls 21-31 lightened it: the probe alternating, 2 rounds; config 5's kernel stats at the default
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_33
mkdir -p $O
for r in 1 2; do
  for b in 4 2 1; do
    timeout -k 10 200 env QDML_QSTREAM_BPB=$b python -u scripts/probes/probe_qstream.py 6 2>&1 | grep n=16 | sed "s/^/bpb=$b /" | tee -a $O/${P}_probe.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --qubits 16 --gradient-pruning --dtype fp8 > $O/${P}_prof.log 2>&1 || { tail -5 $O/${P}_prof.log; exit 1; }
db=$(find $O/${P}_prof -name '*.db' | head -1)
python scripts/prof_summary.py $db --tail 0.6 > $O/${P}_q16_kernel_stats.md 2>&1; head -22 $O/${P}_q16_kernel_stats.md
rm -rf $O/${P}_prof
