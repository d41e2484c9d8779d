#!/bin/bash
# round-5 GPU call 4: the 12-qubit MFMA simulator's numerics (tests/test_qsim12_gpu.py) and its P256 bench against
# the VALU kernels; e4m3 GEMMs with producer waves (numerics, isolated timing, fp8-step A/B against the shipped e4m3
# tiles and the bf16 step), then the kernel timeline of the new default bf16 step (FC GEMM cfg 8,7,6)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qsim12_gpu.py -x -v --timeout 120 --timeout-method thread > $O/r5_04_qsim12_pytest.log 2>&1; tail -15 $O/r5_04_qsim12_pytest.log
grep -q " passed" $O/r5_04_qsim12_pytest.log && ! grep -q "failed\|error" $O/r5_04_qsim12_pytest.log && for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python bench.py --qsim-mfma12 $v --pilot 256 --qubits 12 --steps 100 --warmup 10 > $O/r5_04_cur.json 2> $O/r5_04_cur.err || { tail -20 $O/r5_04_cur.err; exit 1; }
    echo "round $r [p256 q12 mfma12=$v] $(python -c "import json; d=json.load(open('$O/r5_04_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_04_p256.txt
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "f8" --timeout 120 --timeout-method thread > $O/r5_04_pytest.log 2>&1 || { tail -30 $O/r5_04_pytest.log; exit 1; }
tail -2 $O/r5_04_pytest.log
timeout -k 10 300 python scripts/probes/probe_gemm_r5.py 5 fwd8,wgrad8,dgrad8,fwd_c8,wgrad_c7,dgrad_c6 > $O/r5_04_gemm_probe.txt 2>&1; cat $O/r5_04_gemm_probe.txt
for r in 1 2 3; do
  for v in "--dtype bf16" "--dtype fp8 --f8-producers 0" "--dtype fp8 --f8-producers 1"; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 $v > $O/r5_04_cur.json 2> $O/r5_04_cur.err || { tail -20 $O/r5_04_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_04_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_04_ab.txt
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/prof_step.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_step/run_kernel_trace.csv --tail 0.6 > $O/r5_04_step_kernel_stats.md
python scripts/prof_timeline.py $O/prof_step/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r5_04_step_timeline.md; rm -rf $O/prof_step
cat $O/r5_04_step_timeline.md
