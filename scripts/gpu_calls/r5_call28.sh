#!/bin/bash
# round-5 GPU call 28: what the loss epilogue costs the fp8 estimator's forward GEMM (EPI_NMSE vs the plain e4m3
# forward on the same operands, kernel durations from rocprofv3)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nmse -o run -- python $R/scripts/probes/probe_nmse_epi.py 50 > $O/prof_nmse.log 2>&1) || { tail -20 $O/prof_nmse.log; exit 1; }
python - "$O/prof_nmse/run_kernel_stats.csv" > $O/r5_28_nmse_epi_stats.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{float(r["AverageNs"]) / 1e3:9.2f} us avg  {int(r["Calls"]):5d} calls  {r["Name"][:150]}')
PY
rm -rf $O/prof_nmse
cat $O/r5_28_nmse_epi_stats.txt
