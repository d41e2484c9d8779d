#!/bin/bash
# round-4 GPU call: NMSE rows in one round -- numerics + in-step kernel time (compare r4_18_step_kernel_stats.md)
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_flagship_gpu.py -q --timeout 200 --timeout-method thread -k "nmse or bit_exact" > $O/r4_25_pytest.log 2>&1; echo "pytest rc=$?" >> $O/r4_25_pytest.log
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r4_25_bench.json 2>$O/r4_25_bench.err || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/prof_step.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_step/run_kernel_trace.csv --tail 0.6 > $O/r4_25_step_kernel_stats.md; rm -rf $O/prof_step
