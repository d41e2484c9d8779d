#!/bin/bash
# round-5 GPU call 27: the e4m3 data gradient's BN-reduction epilogue re-measured with the unrolled butterfly (r5_21 /
# r5_24 had it at +17 us with the rolled one): isolated probe, then the fp8 step A/B (dgrad_bnred_f8 on / off)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u scripts/probes/probe_gemm_r5.py 7 dgrad8 > $O/r5_27_dgrad8_bnred_probe.txt 2>&1 || { tail -30 $O/r5_27_dgrad8_bnred_probe.txt; exit 1; }
grep median $O/r5_27_dgrad8_bnred_probe.txt
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_27_cur.json 2> $O/r5_27_cur.err || { tail -20 $O/r5_27_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_27_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_27_ab.txt
}
for r in 1 2 3; do
  run "r$r fp8 bnred_f8" --dtype fp8 --knob dgrad_bnred_f8=1
  run "r$r fp8 own_launch" --dtype fp8
done
