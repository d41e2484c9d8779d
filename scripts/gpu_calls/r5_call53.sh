#!/bin/bash
# round-5 GPU call 53: the QSC preprocess forward launched next to one partner kernel on another stream, no graphs
# (scripts/probes/probe_qsc_coresident.py): which partner, if any, makes its results differ from a serial launch
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u scripts/probes/probe_qsc_coresident.py 40 > $O/r5_53_qsc_coresident.txt 2>&1 || { tail -20 $O/r5_53_qsc_coresident.txt; exit 1; }
grep -v "amdgpu.ids" $O/r5_53_qsc_coresident.txt
