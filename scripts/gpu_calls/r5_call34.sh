#!/bin/bash
# round-5 GPU call 35 (call 34 + every QSC buffer after step 1): where the split-forward plans with the fused-loss forward leave the serial step (call 32):
# per-step comparison of the serial reference and the graph plan (scripts/probes/probe_split_fused.py)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
for a in "fwd fcnext" "fwdplain fcnext"; do
  timeout -k 10 200 python -u scripts/probes/probe_split_fused.py $a 1 >> $O/r5_35_split_fused.txt 2>&1 || { tail -20 $O/r5_35_split_fused.txt; exit 1; }
done
grep -v "amdgpu.ids" $O/r5_35_split_fused.txt
