#!/bin/bash
# round-4 GPU call: clock-stamp phase tests, P256 large batch / 16-qubit benches, Adam probe, P256 timeline
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_runtime_gpu.py tests/test_flagship_gpu.py -v --timeout 200 --timeout-method thread -k "clock_stamps or one_graph" > $O/r4_11_stamps.log 2>&1 || exit 1
QDML_FORCE_DIST=1 timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/r4_11_bench_forced_stamps.json 2>$O/r4_11_bench_forced_stamps.err || exit 1
timeout -k 10 300 python bench.py --pilot 256 --qubits 12 --batch 1024 --data-len 60000 --steps 40 --warmup 5 > $O/r4_11_bench_p256_b1024.json 2>$O/r4_11_bench_p256_b1024.err || exit 1
timeout -k 10 300 python bench.py --qubits 16 --dtype fp8 --steps 20 --warmup 3 > $O/r4_11_bench_q16.json 2>$O/r4_11_bench_q16.err || exit 1
timeout -k 10 120 python scripts/probes/r4_adam_probe.py > $O/r4_11_adam_probe.txt 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_p256 -o run -- python $R/bench.py --pilot 256 --qubits 12 --steps 30 --warmup 5 --steps-per-graph 1 > $O/tl_p256.log 2>&1) || exit 1
python scripts/prof_timeline.py $O/tl_p256/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r4_11_p256_timeline.md
python scripts/prof_summary.py $O/tl_p256/run_kernel_trace.csv --tail 0.6 > $O/r4_11_p256_kernel_stats.md; rm -rf $O/tl_p256
timeout -k 10 420 python scripts/probes/r4_conv_sweep.py 300 2 > $O/r4_11_conv_sweep.txt 2>&1 || exit 1
