#!/bin/bash
# round-5 GPU call 48: counters of the final round-5 step (bf16 defaults; one pass per run): MFMA busy, LDS traffic /
# bank conflicts, HBM bytes and L2 hits per kernel, and the same for the isolated FC GEMMs (probe_gemm_r5.py)
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
P3="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P4="TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum"
TAG=r5_48 PASSES="FETCH_SIZE;WRITE_SIZE;$P3;$P4" bash scripts/gpu_calls/r4_pmc.sh || exit 1
CMD="$R/scripts/probes/probe_gemm_r5.py 3 fwd_c8,wgrad_c7,dgrad_c6,dgrad_bnred_c6" TAG=r5_48iso PASSES="FETCH_SIZE;$P3" bash scripts/gpu_calls/r4_pmc.sh || exit 1
head -30 $O/r5_48_pmc_summary.md | cut -c1-220
