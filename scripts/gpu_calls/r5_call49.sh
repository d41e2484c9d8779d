#!/bin/bash
# round-5 GPU call 49: the fp8 estimator's e4m3 convs (KNOBS.fp8_conv, layers 2 / 3) re-measured on the final tree,
# step A/B against the default fp8 step, 3 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_49_cur.json 2> $O/r5_49_cur.err || { tail -20 $O/r5_49_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_49_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_49_ab.txt
}
for r in 1 2 3; do
  run "r$r fp8" --dtype fp8
  run "r$r fp8 + e4m3 convs" --dtype fp8 --knob fp8_conv=1
  run "r$r bf16"
done
