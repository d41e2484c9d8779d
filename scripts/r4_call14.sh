#!/bin/bash
# round-4 GPU call: captured-RCCL regression check (inline small bucket, ordering without duplicate waits)
cd "$(dirname "$0")/.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_comm_gpu.py tests/test_flagship_gpu.py -v --timeout 200 --timeout-method thread -k "rccl or one_graph" > $O/r4_14_pytest.log 2>&1 || exit 1
QDML_FORCE_DIST=1 timeout -k 10 400 python bench.py --steps 200 --warmup 20 --select-steps 30 > $O/r4_14_bench_forced.json 2>$O/r4_14_bench_forced.err || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r4_14_pytest_full.log 2>&1; echo "pytest rc=$?" >> $O/r4_14_pytest_full.log
