#!/bin/bash
# round-5 GPU call 5: e4m3 GEMMs with producer waves (numerics, isolated timing, fp8-step A/B against the shipped
# e4m3 tiles and the bf16 step); kernel timelines of the new default bf16 step and of the P256 / 12-qubit step on
# the MFMA simulator
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "f8" --timeout 120 --timeout-method thread > $O/r5_05_pytest.log 2>&1 || { tail -30 $O/r5_05_pytest.log; exit 1; }
tail -2 $O/r5_05_pytest.log
timeout -k 10 300 python scripts/probes/probe_gemm_r5.py 5 fwd8,wgrad8,dgrad8,fwd_c8,wgrad_c7,dgrad_c6 > $O/r5_05_gemm_probe.txt 2>&1; cat $O/r5_05_gemm_probe.txt
for r in 1 2 3; do
  for v in "--dtype bf16" "--dtype fp8 --f8-producers 0" "--dtype fp8 --f8-producers 1"; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 $v > $O/r5_05_cur.json 2> $O/r5_05_cur.err || { tail -20 $O/r5_05_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_05_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_05_ab.txt
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/prof_step.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_step/run_kernel_trace.csv --tail 0.6 > $O/r5_05_step_kernel_stats.md
python scripts/prof_timeline.py $O/prof_step/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r5_05_step_timeline.md; rm -rf $O/prof_step
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p256 -o run -- python $R/bench.py --pilot 256 --qubits 12 --steps 40 --warmup 10 > $O/prof_p256.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_p256/run_kernel_trace.csv --tail 0.6 > $O/r5_05_p256_kernel_stats.md
python scripts/prof_timeline.py $O/prof_p256/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r5_05_p256_timeline.md; rm -rf $O/prof_p256
cat $O/r5_05_step_timeline.md $O/r5_05_p256_timeline.md
head -20 $O/r5_05_p256_kernel_stats.md
