#!/bin/bash
# round-4 GPU call (diagnostic): the HDCE chain alone and the QSC branch alone vs the shipped step, + timelines
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
ROUNDS=2 PLAN=shipped,hdce_only,qsc_only timeout -k 10 400 python scripts/probes/r4_plan_probe.py 400 > $O/r4_22_plans.txt 2>&1 || exit 1
for p in hdce_only qsc_only; do
  (cd /tmp && export TMPDIR=/tmp && PLAN=$p timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$p -o run -- python $R/scripts/probes/r4_plan_probe.py 100 > $O/tl_$p.log 2>&1) || exit 1
  python scripts/prof_summary.py $O/tl_$p/run_kernel_trace.csv --tail 0.6 > $O/r4_22_stats_$p.md; rm -rf $O/tl_$p
done
