#!/bin/bash
# round-5 GPU call 37: does the QSC forward of the split-forward plan (fc_adam_next) with the fused-loss forward read
# the classifier input before its gather wrote it?  xq poisoned with NaN before each replay
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
PROBE_POISON_XQ=1 timeout -k 10 200 python -u scripts/probes/probe_split_fused.py fwd fcnext 2 > $O/r5_37_poison_xq.txt 2>&1 || { tail -20 $O/r5_37_poison_xq.txt; exit 1; }
grep -v "amdgpu.ids\|OVERLAP\|   cstep.hip.w2t\|   cstep.hip.q\|   cstep.hip._w\|   cstep.hip.noise\|   cstep.skip\|   cstep.hip.psave" $O/r5_37_poison_xq.txt
