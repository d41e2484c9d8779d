#!/bin/bash
# round-5 GPU call 18: full GPU suite on the current tree; the persistent conv forward with one workgroup per CU
# (spw 3: 198 workgroups -- its stamps showed doubled-up CUs' workgroups gating every barrier) against the default
# and the per-layer spw 3, 2 alternating rounds; the driver's 20-step window
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5_18_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/r5_18_pytest.log
tail -3 $O/r5_18_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_18_cur.json 2> $O/r5_18_cur.err || { tail -20 $O/r5_18_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_18_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_18_ab.txt
}
for r in 1 2; do
  run "r$r default"
  run "r$r spw3" --knob conv_spw=3
  run "r$r stack_spw3" --knob conv_stack=1 --knob conv_spw=3
  run "r$r stack_spw4" --knob conv_stack=1 --knob conv_spw=4
done
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/r5_18_cur.json 2> $O/r5_18_cur.err || exit 1
  echo "[window r$r] $(python -c "import json; d=json.load(open('$O/r5_18_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['replays'])")" | tee -a $O/r5_18_ab.txt
done
