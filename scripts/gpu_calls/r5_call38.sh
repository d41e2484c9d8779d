#!/bin/bash
# round-5 GPU call 38: the split-forward + fused-loss QSC mismatch -- recompute the QSC preprocess forward eagerly
# from each side's pre-step weights and compare with what its step produced
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
PROBE_RECOMPUTE=1 timeout -k 10 200 python -u scripts/probes/probe_split_fused.py fwd fcnext 1 > $O/r5_38_recompute.txt 2>&1 || { tail -20 $O/r5_38_recompute.txt; exit 1; }
grep -v "amdgpu.ids\|OVERLAP\|   cstep.hip.w2t\|   cstep.hip.q\|   cstep.hip._w\|   cstep.hip.noise\|   cstep.skip\|   cstep.hip.psave" $O/r5_38_recompute.txt
