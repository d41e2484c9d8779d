cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for r in 1 2; do
  timeout -k 10 60 python $R/scripts/probe_conv_bwd.py --fused 0 --iters 40 >> $O/probe.log 2>&1 || exit 1
  for s in 3 4 5 6 8; do timeout -k 10 60 python $R/scripts/probe_conv_bwd.py --fused 1 --spb-f $s --iters 40 >> $O/probe.log 2>&1 || exit 1; done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_1 -o run -- python $R/scripts/probe_conv_bwd.py --iters 20 > $O/kt_1.log 2>&1 || exit 1
