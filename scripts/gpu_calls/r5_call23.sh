#!/bin/bash
# round-5 GPU call 23: the data gradients alone with / without layer 3's BN backward reduction in the epilogue (bf16
# cfg 6, e4m3 cfg 0 / 1): r5_22 put the e4m3 one at 50 us in the step against 33 without
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u scripts/probes/probe_gemm_r5.py 7 dgrad > $O/r5_23_dgrad_bnred_probe.txt 2>&1 || { tail -30 $O/r5_23_dgrad_bnred_probe.txt; exit 1; }
cat $O/r5_23_dgrad_bnred_probe.txt
