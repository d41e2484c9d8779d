#!/bin/bash
# round-5 GPU call 52: call 38 again (fcnext and conv) with the differing samples of the graph run listed by workgroup and XCD
# (a per-XCD pattern would point at stale L2 lines)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
for m in fcnext conv; do PROBE_RECOMPUTE=1 timeout -k 10 200 python -u scripts/probes/probe_split_fused.py wgrad $m 1 >> $O/r5_52_recompute_xcd.txt 2>&1 || { tail -20 $O/r5_52_recompute_xcd.txt; exit 1; }; done
grep "differ\|recompute\|^step\|^\[" $O/r5_52_recompute_xcd.txt; true #   cstep.hip.w2t\|   cstep.hip.q\|   cstep.hip._w\|   cstep.hip.noise\|   cstep.skip\|   cstep.hip.psave" $O/r5_52_recompute_xcd.txt
