#!/bin/bash
# round-5 GPU call 44: the QSC preprocess forward on fewer workgroups (KNOBS.qsc_fwd_cap 128 / 64, default 256) so the
# FC forward's 136-KB workgroups find free CUs at once (r5_33's timeline: a 14 us wait), step A/B, 3 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_44_cur.json 2> $O/r5_44_cur.err || { tail -20 $O/r5_44_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_44_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_44_ab.txt
}
for r in 1 2 3; do
  run "r$r cap 256"
  run "r$r cap 128" --knob qsc_fwd_cap=128
  run "r$r cap 64" --knob qsc_fwd_cap=64
done
