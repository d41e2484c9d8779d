#!/bin/bash
# round-5 GPU call 10: stream_mode "indep" (QSC and HDCE chains independent for the whole replay, each with its own
# gather: no cross-queue edge on the HDCE chain): bit-exactness against the serial eager step, then the step A/B
# against dagq; then the conv stack's launch shapes (knobs conv_spw / conv_spb_f / conv_spb_w1) in the step
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_flagship_gpu.py -x -q -k "multistream or bit_exact" --timeout 200 --timeout-method thread > $O/r5_10_pytest.log 2>&1 || { tail -40 $O/r5_10_pytest.log; exit 1; }
tail -2 $O/r5_10_pytest.log
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_10_cur.json 2> $O/r5_10_cur.err || { tail -20 $O/r5_10_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_10_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_10_ab.txt
}
for r in 1 2; do
  run "r$r dagq" --stream-mode dagq
  run "r$r indep" --stream-mode indep
done
for r in 1 2; do
  run "r$r base"
  run "r$r spw1" --knob conv_spw=1
  run "r$r spw3" --knob conv_spw=3
  run "r$r spw4" --knob conv_spw=4
  run "r$r spbf4" --knob conv_spb_f=4
  run "r$r spbf6" --knob conv_spb_f=6
  run "r$r spbf8" --knob conv_spb_f=8
  run "r$r spbw1_2" --knob conv_spb_w1=2
  run "r$r spbw1_8" --knob conv_spb_w1=8
done
