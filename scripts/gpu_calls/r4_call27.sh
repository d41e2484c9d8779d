#!/bin/bash
# conv VALU diet (packed BN/ReLU staging, packed epilogue statistics, permlane32 stores): conv tests, an A/B of
# the step against the previous library (lib_ab/libqdml_hip_base.so swapped in), and the new step's kernel stats
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; L=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_kernels_gpu.py tests/test_flagship_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r4_27_pytest.log 2>&1 || exit 1
cp $L/libqdml_hip.so $R/lib_ab/libqdml_hip_new.so
for r in 0 1; do
  for v in new base; do
    cp $R/lib_ab/libqdml_hip_$v.so $L/libqdml_hip.so
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 > $O/r4_27_bench_${v}_$r.json 2>$O/r4_27_bench_${v}_$r.err || exit 1
    echo "round $r $v $(python -c "import json,sys; d=json.load(open('$O/r4_27_bench_${v}_$r.json')); print(d['ms_per_step'])")" >> $O/r4_27_ab.txt
  done
done
cp $R/lib_ab/libqdml_hip_new.so $L/libqdml_hip.so
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/prof_step.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_step/run_kernel_trace.csv --tail 0.6 > $O/r4_27_step_kernel_stats.md
python scripts/prof_timeline.py $O/prof_step/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r4_27_step_timeline.md; rm -rf $O/prof_step
