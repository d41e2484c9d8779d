cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for v in "" "--f32"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/q$v -o run -- python $R/scripts/probe_qsc_bwd.py --iters 20 $v > $O/q$v.log 2>&1 || exit 1
done
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmcq -o run -- python $R/scripts/probe_qsc_bwd.py --iters 6 > $O/pmcq.log 2>&1 || exit 1
