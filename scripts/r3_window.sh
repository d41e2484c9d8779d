#!/bin/bash
# Round-3 baseline: the driver's exact short window (--steps 20 --warmup 5) and a long window back to
# back on one box, repeated, plus the isolated FC GEMM probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2; do
  for a in "--steps 20 --warmup 5" "--steps 300 --warmup 10"; do
    timeout -k 10 300 python bench.py $a > $OUT/w.log 2>&1 || { tail -20 $OUT/w.log; exit 1; }
    echo "round $r [$a] $(grep -o '"ms_per_step": [0-9.]*' $OUT/w.log) $(grep -o '"host_ms_per_step": [0-9.]*' $OUT/w.log)" | tee -a $OUT/r3_window.txt
  done
done
timeout -k 10 300 python scripts/probe_gemm.py > $OUT/r3_probe_gemm.log 2>&1 || { tail -20 $OUT/r3_probe_gemm.log; exit 1; }
cat $OUT/r3_probe_gemm.log
