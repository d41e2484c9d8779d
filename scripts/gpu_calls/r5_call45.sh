#!/bin/bash
# round-5 GPU call 45: the loss epilogue's coefficient loads 4 rows per lane in flight and the next batch's row offsets
# loaded ahead (no barrier changes; the direct-A tile keeps the old code): NMSE / GEMM / fp8 tests, the epilogue
# probe, fp8 step A/B against the previous library (3 rounds)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
L=quantum_distributed_machine_learning_ris_channel_estimation_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_conv_gpu.py tests/test_flagship_gpu.py -x -q -k "nmse or fp8 or f8 or loss or bit_exact or hand_gemm" --timeout 200 --timeout-method thread > $O/r5_45_pytest.log 2>&1 || { tail -40 $O/r5_45_pytest.log; exit 1; }
tail -1 $O/r5_45_pytest.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nmse -o run -- python $R/scripts/probes/probe_nmse_epi.py 50 > $O/prof_nmse.log 2>&1) || { tail -20 $O/prof_nmse.log; exit 1; }
python - "$O/prof_nmse/run_kernel_stats.csv" > $O/r5_45_nmse_epi_stats.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:3]:
    print(f'{float(r["AverageNs"]) / 1e3:9.2f} us avg  {int(r["Calls"]):5d} calls  {r["Name"][:150]}')
PY
rm -rf $O/prof_nmse
cat $O/r5_45_nmse_epi_stats.txt
cp $L/libqdml_hip.so $O/new.so
run() {   # label, lib, bench args...
  local lab=$1 lib=$2; shift 2
  cp $lib $L/libqdml_hip.so
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_45_cur.json 2> $O/r5_45_cur.err || { tail -20 $O/r5_45_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_45_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_45_ab.txt
}
for r in 1 2 3; do
  run "r$r fp8 new" $O/new.so --dtype fp8
  run "r$r fp8 base" $L/libqdml_hip_base.so --dtype fp8
done
cp $O/new.so $L/libqdml_hip.so && rm -f $O/new.so
