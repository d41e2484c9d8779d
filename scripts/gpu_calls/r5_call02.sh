#!/bin/bash
# round-5 GPU call 2: the driver's window on a FRESH box (bench first, nothing before it), default settle (30 steps)
# vs a long settle (300 untimed steps), alternating; then the producer-wave GEMM probe
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out
for r in 1 2; do
  for v in "--settle-steps 30" "--settle-steps 300"; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 $v > $O/r5_02_cur.json 2> $O/r5_02_cur.err || { tail -20 $O/r5_02_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_02_cur.json')); print(d['ms_per_step'], d['step_spread'])")" | tee -a $O/r5_02_window.txt
  done
done
timeout -k 10 300 python scripts/probes/probe_gemm_r5.py 5 > $O/r5_02_gemm_probe.txt 2>&1; cat $O/r5_02_gemm_probe.txt
# the FC weight's Adam beside the conv backward (--fc-adam-side N workgroups) vs at the tail, 2 rounds, --steps 300
for r in 1 2; do
  for v in "--fc-adam-side 0" "--fc-adam-side 64" "--fc-adam-side 128" "--fc-adam-side 256"; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 $v > $O/r5_02_cur.json 2> $O/r5_02_cur.err || { tail -20 $O/r5_02_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_02_cur.json')); print(d['ms_per_step'], d['step_spread'], d['config']['fc_adam_side'])")" | tee -a $O/r5_02_adam_side.txt
  done
done
