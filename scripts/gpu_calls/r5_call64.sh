#!/bin/bash
# round-5 GPU call 64: conv1 k-loop unrolled 3 (weights now in SGPRs) in the QSC preprocess forward: bf16 default
# step A/B against the previous qsc_mfma.hip (lib/libqdml_hip_base.so, scripts/build_ab_lib.sh 7673643 qsc_mfma.hip), 4 rounds (a second box)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
L=quantum_distributed_machine_learning_ris_channel_estimation_amd/lib
NEW=/tmp/qd_new_$$.so
cp $L/libqdml_hip.so $NEW
run() {   # label, lib, bench args...
  local lab=$1 lib=$2; shift 2
  cp $lib $L/libqdml_hip.so
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_64_cur.json 2> $O/r5_64_cur.err || { tail -20 $O/r5_64_cur.err; cp $NEW $L/libqdml_hip.so; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_64_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_64_ab.txt
}
for r in 1 2 3 4; do
  run "r$r bf16 unroll3" $NEW
  run "r$r bf16 base" $L/libqdml_hip_base.so
done
cp $NEW $L/libqdml_hip.so && rm -f $NEW $O/r5_64_cur.json $O/r5_64_cur.err
