#!/bin/bash
# Round 3: CU partitions that leave every XCD some CUs (logical CU bit b -> XCD b % 8, then SE, then CU).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
STEPS=variants BENCH_STEPS=200 VARIANTS="${VARIANTS:-NONE=0|--no-graphs;QDML_QSC_CUS=0-255|--no-graphs;QDML_QSC_CUS=0-255 QDML_MAIN_CUS=0-255|--no-graphs;QDML_QSC_CUS=first:32 QDML_MAIN_CUS=32-255|--no-graphs;QDML_QSC_CUS=first:64 QDML_MAIN_CUS=64-255|--no-graphs;QDML_QSC_CUS=first:96 QDML_MAIN_CUS=96-255|--no-graphs;QDML_QSC_CUS=first:128 QDML_MAIN_CUS=128-255|--no-graphs;QDML_QSC_CUS=first:64|--no-graphs;QDML_QSC_CUS=first:64 QDML_MAIN_CUS=64-255|}" bash scripts/gpu_check.sh || exit 1
