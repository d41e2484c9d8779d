#!/bin/bash
# round-5 GPU call 30: the loss epilogue's global reads prefetched (label powers + first batch's row offsets before
# the fp32 tile's LDS round, LDS-only barriers; every batch's offsets up front, labels one batch ahead): tests,
# epilogue probe, fp8 and bf16 step A/B against the previous library.
# RESULT: the direct-A tile (cfg 5) faulted in test_gemm_nmse_epilogue_matches_fp32 (profiles/r5_30_prefetch_fault_pytest.log);
# the change was reverted (gemm.hip as of the call-29 tree) -- cause not found by inspection
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
L=quantum_distributed_machine_learning_ris_channel_estimation_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_conv_gpu.py tests/test_flagship_gpu.py -x -q -k "nmse or fp8 or f8 or loss or bit_exact or hand_gemm" --timeout 200 --timeout-method thread > $O/r5_30_pytest.log 2>&1 || { tail -40 $O/r5_30_pytest.log; exit 1; }
tail -1 $O/r5_30_pytest.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nmse -o run -- python $R/scripts/probes/probe_nmse_epi.py 50 > $O/prof_nmse.log 2>&1) || { tail -20 $O/prof_nmse.log; exit 1; }
python - "$O/prof_nmse/run_kernel_stats.csv" > $O/r5_30_nmse_epi_stats.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:3]:
    print(f'{float(r["AverageNs"]) / 1e3:9.2f} us avg  {int(r["Calls"]):5d} calls  {r["Name"][:150]}')
PY
rm -rf $O/prof_nmse
cat $O/r5_30_nmse_epi_stats.txt
cp $L/libqdml_hip.so $O/new.so
run() {   # label, lib, bench args...
  local lab=$1 lib=$2; shift 2
  cp $lib $L/libqdml_hip.so
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_30_cur.json 2> $O/r5_30_cur.err || { tail -20 $O/r5_30_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_30_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_30_ab.txt
}
for r in 1 2; do
  run "r$r fp8 prefetch" $O/new.so --dtype fp8
  run "r$r fp8 base" $L/libqdml_hip_base.so --dtype fp8
  run "r$r bf16 prefetch" $O/new.so
  run "r$r bf16 base" $L/libqdml_hip_base.so
done
cp $O/new.so $L/libqdml_hip.so && rm -f $O/new.so
