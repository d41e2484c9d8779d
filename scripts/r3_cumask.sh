#!/bin/bash
# Round 3: CU-masked streams -- does the mask hold (eager / graph replay), and does partitioning the
# chip between the QSC branch and the HDCE chain beat the dispatcher's first-come placement?
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 180 python scripts/probe_cumask.py > $OUT/cumask_probe.log 2>&1 || { tail -30 $OUT/cumask_probe.log; exit 1; }
cat $OUT/cumask_probe.log
Q64="stride:4:0"; M192="stride:4:1+stride:4:2+stride:4:3"
Q32="stride:8:0"; M224="stride:8:1+stride:8:2+stride:8:3+stride:8:4+stride:8:5+stride:8:6+stride:8:7"
STEPS=variants BENCH_STEPS=200 VARIANTS="NONE=0|;NONE=0|--no-graphs;QDML_QSC_CUS=$Q64|--no-graphs;QDML_QSC_CUS=$Q64 QDML_MAIN_CUS=$M192|--no-graphs;QDML_QSC_CUS=$Q32 QDML_MAIN_CUS=$M224|--no-graphs;QDML_QSC_CUS=$Q64 QDML_MAIN_CUS=$M192|" bash scripts/gpu_check.sh || exit 1
