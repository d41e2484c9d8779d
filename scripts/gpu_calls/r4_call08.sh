#!/bin/bash
# round-4 GPU call: step-plan probe + timelines, the GEMM probe, in-step and isolated GEMM counters
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_flagship_gpu.py -q --timeout 120 --timeout-method thread -k two_ranks > $O/r4_08_pytest.log 2>&1; echo "pytest rc=$?" >> $O/r4_08_pytest.log
timeout -k 10 300 python scripts/probes/r4_plan_probe.py 300 > $O/r4_08_plans.txt 2>&1 || exit 1
for p in hdce_first join_first; do
  (cd /tmp && export TMPDIR=/tmp && PLAN=$p timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$p -o run -- python $R/scripts/probes/r4_plan_probe.py 100 > $O/tl_$p.log 2>&1) || exit 1
  python scripts/prof_timeline.py $O/tl_$p/run_kernel_trace.csv --marker "conv3x3_kernel<2," > $O/r4_08_timeline_$p.md; rm -rf $O/tl_$p
done
timeout -k 10 300 python scripts/probes/probe_gemm.py > $O/r4_08_gemm_probe.txt 2>&1 || exit 1
P3="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P4="TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum"
TAG=r4_08 PASSES="FETCH_SIZE;WRITE_SIZE;$P3;$P4" bash scripts/gpu_calls/r4_pmc.sh || exit 1
PROBE_ONLY=fwd_hand1,wgrad_hand1,dgrad_hand2_1x8,fwd_hand1_cold,flush_only CMD="$R/scripts/probes/probe_gemm.py" TAG=r4_08iso PASSES="FETCH_SIZE;$P3;$P4" bash scripts/gpu_calls/r4_pmc.sh
