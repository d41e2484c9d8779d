cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for r in 1 2; do
  timeout -k 10 60 python $R/scripts/probe_conv_bwd.py --fused 0 --iters 40 >> $O/probe.log 2>&1 || exit 1
  for s in 4 5 6 8; do timeout -k 10 60 python $R/scripts/probe_conv_bwd.py --fused 1 --spb-f $s --iters 40 >> $O/probe.log 2>&1 || exit 1; done
done
cd $R
for i in 1 2; do timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b$i.log 2>&1 || exit 1; QDML_CONV_BWD_FUSED=0 timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/c$i.log 2>&1 || exit 1; done
