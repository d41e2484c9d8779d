#!/bin/bash
# round-5 GPU call 55: the differing p1s entries of the graph run (window, channel, values), and the xq poison
# check (NaN before the replay) with the hipBLASLt forward
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
PROBE_RECOMPUTE=1 timeout -k 10 200 python -u scripts/probes/probe_split_fused.py wgrad fcnext 1 > $O/r5_55_entries.txt 2>&1 || { tail -20 $O/r5_55_entries.txt; exit 1; }
PROBE_RECOMPUTE=1 PROBE_POISON_XQ=1 timeout -k 10 200 python -u scripts/probes/probe_split_fused.py wgrad fcnext 1 >> $O/r5_55_entries.txt 2>&1 || { tail -20 $O/r5_55_entries.txt; exit 1; }
grep "differ\|recompute\|^step\|^\[\|sample" $O/r5_55_entries.txt; true
