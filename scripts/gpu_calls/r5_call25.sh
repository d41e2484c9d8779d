#!/bin/bash
# round-5 GPU call 25: where the bf16 data gradient's BN-reduction epilogue spends its +9 us (diagnosis variants: no z
# loads / no cross-lane reduction / neither), isolated
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u scripts/probes/probe_gemm_r5.py 7 dgrad_c6,dgrad_bnred > $O/r5_25_dgrad_bnred_dbg.txt 2>&1 || { tail -30 $O/r5_25_dgrad_bnred_dbg.txt; exit 1; }
cat $O/r5_25_dgrad_bnred_dbg.txt
