#!/bin/bash
# round-5 GPU call 39: the split-forward + fused-loss QSC mismatch -- buffer overlap check incl. the parameter spaces,
# optimizer moments and the conv stack's buffer lists
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
PROBE_X=1 timeout -k 10 200 python -u scripts/probes/probe_split_fused.py fwd fcnext 1 > $O/r5_39_overlap.txt 2>&1 || { tail -20 $O/r5_39_overlap.txt; exit 1; }
grep -v "amdgpu.ids\|   cstep.hip.w2t\|   cstep.hip.q\|   cstep.hip._w\|   cstep.hip.noise\|   cstep.skip\|   cstep.hip.psave" $O/r5_39_overlap.txt
