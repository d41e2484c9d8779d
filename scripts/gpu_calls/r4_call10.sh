#!/bin/bash
# round-4 GPU call: GEMM config tests + timings, QSC HIP validation test, P256 / 16-qubit benches + P256 timeline
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_qsc_gpu.py -q --timeout 120 --timeout-method thread -k "matches_fp32 or validation" > $O/r4_10_pytest.log 2>&1; echo "pytest rc=$?" >> $O/r4_10_pytest.log
PROBE_ONLY=fwd_hand0,fwd_hand1,fwd_hand2_ks2,fwd_hand3_4x1,fwd_hand4_2x2,fwd_hand5_directA,wgrad_hand1,wgrad_hand3_2x2,dgrad_hand2_1x8,dgrad_hand4_288,fwd_hipblaslt timeout -k 10 300 python scripts/probes/probe_gemm.py > $O/r4_10_gemm_probe.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --pilot 256 --qubits 12 --steps 100 --warmup 10 > $O/r4_10_bench_p256.json 2>$O/r4_10_bench_p256.err || exit 1
timeout -k 10 300 python bench.py --pilot 256 --qubits 12 --batch 1024 --steps 40 --warmup 5 > $O/r4_10_bench_p256_b1024.json 2>$O/r4_10_bench_p256_b1024.err || exit 1
timeout -k 10 300 python bench.py --qubits 16 --dtype fp8 --steps 20 --warmup 3 > $O/r4_10_bench_q16.json 2>$O/r4_10_bench_q16.err || exit 1
timeout -k 10 120 python scripts/probes/r4_adam_probe.py > $O/r4_10_adam_probe.txt 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_p256 -o run -- python $R/bench.py --pilot 256 --qubits 12 --steps 30 --warmup 5 --steps-per-graph 1 > $O/tl_p256.log 2>&1) || exit 1
python scripts/prof_timeline.py $O/tl_p256/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r4_10_p256_timeline.md
python scripts/prof_summary.py $O/tl_p256/run_kernel_trace.csv --tail 0.6 > $O/r4_10_p256_kernel_stats.md; rm -rf $O/tl_p256
VARIANTS="N=0|;N=1|--gemm-cfg 3,1,2;N=2|--gemm-cfg 5,1,2;N=3|--gemm-cfg 1,3,4" bash scripts/gpu_calls/r4_ab.sh $O/r4_10_gemm_cfg_ab.txt || exit 1
timeout -k 10 400 python -u -m pytest tests/test_runtime_gpu.py tests/test_flagship_gpu.py -v --timeout 200 --timeout-method thread -k "clock_stamps or one_graph" > $O/r4_10_stamps.log 2>&1 || exit 1
QDML_FORCE_DIST=1 timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/r4_10_bench_forced_stamps.json 2>$O/r4_10_bench_forced_stamps.err
