#!/bin/bash
# round-5 GPU call 41: the split-forward + fused-loss QSC mismatch -- the device buffer address map
# (which allocations sit next to the QSC weights and inputs)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
PROBE_MAP=1 timeout -k 10 200 python -u scripts/probes/probe_split_fused.py fwd fcnext 1 > $O/r5_41_map.txt 2>&1 || { tail -20 $O/r5_41_map.txt; exit 1; }
grep -v "amdgpu.ids\|   cstep.hip.w2t\|   cstep.hip.q\|   cstep.hip._w\|   cstep.hip.noise\|   cstep.skip\|   cstep.hip.psave" $O/r5_41_map.txt
