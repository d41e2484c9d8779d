#!/bin/bash
# round-6 GPU call 60: (after call 55: b128 tile accesses, no SI load/store pairing) the streamed 16-qubit simulator alone (probe_qstream.py: forward + adjoint at 2,304 samples),
# timed; then PMC counters of its kernels in two passes of their own
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_60
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/probes/probe_qstream.py 6 > $O/${P}_probe.txt 2>&1 || { tail -5 $O/${P}_probe.txt; exit 1; }
cat $O/${P}_probe.txt
pass() { n=$1; shift; (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/${P}_pmc_$n -o run -- python3 $R/scripts/probes/probe_qstream.py 2 > $O/${P}_pmc_$n.log 2>&1) || { echo "pass $n failed"; tail -5 $O/${P}_pmc_$n.log; return 1; }; }
pass a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS || exit 1
python scripts/pmc_summary.py $O/${P}_pmc_a > $O/${P}_pmc_a.md; grep "qstream" $O/${P}_pmc_a.md | cut -c1-330; head -1 $O/${P}_pmc_a.md
pass b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE FETCH_SIZE || exit 1
python scripts/pmc_summary.py $O/${P}_pmc_b > $O/${P}_pmc_b.md; grep "qstream" $O/${P}_pmc_b.md | cut -c1-330; head -1 $O/${P}_pmc_b.md
rm -rf $O/${P}_pmc_a $O/${P}_pmc_b
