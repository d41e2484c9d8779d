#!/bin/bash
# round-6 GPU call 19: PMC counters of the P128 forward stack on conv3x3_kernel vs conv3x3_split_kernel (sps 5), two
# passes of their own (counter runs only kernel-trace-free collection), summarised per kernel
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_19
mkdir -p $O
export TMPDIR=/tmp
pass() { n=$1; shift; (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/${P}_pmc_$n -o run -- python3 $R/scripts/probes/probe_conv_split.py 10 128 0,5 > $O/${P}_pmc_$n.log 2>&1) || { echo "pass $n failed"; tail -5 $O/${P}_pmc_$n.log; return 1; }; }
pass a SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE || exit 1
python scripts/pmc_summary.py $O/${P}_pmc_a > $O/${P}_pmc_a.md; grep "conv3x3" $O/${P}_pmc_a.md | cut -c1-400; head -2 $O/${P}_pmc_a.md
pass b SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR || exit 1
python scripts/pmc_summary.py $O/${P}_pmc_b > $O/${P}_pmc_b.md; grep "conv3x3" $O/${P}_pmc_b.md | cut -c1-400; head -2 $O/${P}_pmc_b.md
rm -rf $O/${P}_pmc_a $O/${P}_pmc_b
