#!/bin/bash
# round-5 GPU call 24: the e4m3 data gradient's BN reduction run by its producer waves (gemm.hip EPI_BF16_BNP: z
# prefetched during the K loop's last steps; r5_23 had the compute waves' epilogue at +17 us) -- bnred / fp8 tests,
# the isolated probe, the fp8 step A/B
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_gemm_gpu.py -x -q -k "bn_reduction or fp8 or f8" --timeout 200 --timeout-method thread > $O/r5_24_pytest.log 2>&1 || { tail -40 $O/r5_24_pytest.log; exit 1; }
tail -1 $O/r5_24_pytest.log
timeout -k 10 300 python -u scripts/probes/probe_gemm_r5.py 7 dgrad > $O/r5_24_dgrad_bnred_probe.txt 2>&1 || { tail -30 $O/r5_24_dgrad_bnred_probe.txt; exit 1; }
grep median $O/r5_24_dgrad_bnred_probe.txt
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_24_cur.json 2> $O/r5_24_cur.err || { tail -20 $O/r5_24_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_24_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_24_ab.txt
}
for r in 1 2 3; do
  run "r$r fp8 dgrad_bnred" --dtype fp8
  run "r$r fp8 own_launch" --dtype fp8 --knob dgrad_bnred=0
done
