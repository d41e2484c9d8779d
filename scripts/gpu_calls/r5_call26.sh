#!/bin/bash
# round-5 GPU call 26: the BN-reduction epilogue's butterfly unrolled (12 sums side by side; r5_25 put 6 of its 9 us
# in the reduction): the bnred tests, the isolated probe (incl. the diagnosis variants), the bf16 step A/B against
# the previous library (scripts/build_ab_lib.sh -> lib/libqdml_hip_base.so)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
L=quantum_distributed_machine_learning_ris_channel_estimation_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_flagship_gpu.py -x -q -k "bn_reduction or bit_exact" --timeout 200 --timeout-method thread > $O/r5_26_pytest.log 2>&1 || { tail -40 $O/r5_26_pytest.log; exit 1; }
tail -1 $O/r5_26_pytest.log
timeout -k 10 300 python -u scripts/probes/probe_gemm_r5.py 7 dgrad_c6,dgrad_bnred > $O/r5_26_dgrad_bnred_probe.txt 2>&1 || { tail -30 $O/r5_26_dgrad_bnred_probe.txt; exit 1; }
grep median $O/r5_26_dgrad_bnred_probe.txt
cp $L/libqdml_hip.so $O/new.so
run() {   # label, lib, bench args...
  local lab=$1 lib=$2; shift 2
  cp $lib $L/libqdml_hip.so
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_26_cur.json 2> $O/r5_26_cur.err || { tail -20 $O/r5_26_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_26_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_26_ab.txt
}
for r in 1 2 3; do
  run "r$r unrolled" $O/new.so
  run "r$r rolled" $L/libqdml_hip_base.so
done
cp $O/new.so $L/libqdml_hip.so && rm -f $O/new.so
