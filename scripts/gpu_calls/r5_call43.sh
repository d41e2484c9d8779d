#!/bin/bash
# round-5 GPU call 43: the FC forward on a 3-stage ring (cfg 11, 102 KB of LDS: fits beside a QSC preprocess
# workgroup; r5_33's timeline had the forward wait 14 us for that kernel to leave the CUs): GEMM tests, the isolated
# probe, step A/B gemm_cfg 11,7,6 vs 8,7,6 (3 rounds) and a timeline of the new default candidate
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "fwd or nmse" --timeout 200 --timeout-method thread > $O/r5_43_pytest.log 2>&1 || { tail -40 $O/r5_43_pytest.log; exit 1; }
tail -1 $O/r5_43_pytest.log
timeout -k 10 300 python -u scripts/probes/probe_gemm_r5.py 7 fwd_c8,fwd_c11 > $O/r5_43_fwd_probe.txt 2>&1 || { tail -30 $O/r5_43_fwd_probe.txt; exit 1; }
grep median $O/r5_43_fwd_probe.txt
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_43_cur.json 2> $O/r5_43_cur.err || { tail -20 $O/r5_43_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_43_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_43_ab.txt
}
for r in 1 2 3; do
  run "r$r cfg 11,7,6" --gemm-cfg 11,7,6
  run "r$r cfg 8,7,6"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- python $R/bench.py --steps 100 --warmup 20 --gemm-cfg 11,7,6 > $O/prof_step.log 2>&1) || exit 1
python scripts/prof_timeline.py $O/prof_step/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r5_43_step_timeline.md; rm -rf $O/prof_step
head -16 $O/r5_43_step_timeline.md
