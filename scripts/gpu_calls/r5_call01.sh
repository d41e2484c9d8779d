#!/bin/bash
# round-5 GPU call 1: full GPU suite on the round-5 tree (watchdog on), then the driver's window (--steps 20
# --warmup 5) with the replay ramp vs without (--ramp 0), alternating 3 rounds, then --steps 300
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r5_01_pytest.log 2>&1 || { tail -30 $O/r5_01_pytest.log; exit 1; }
tail -3 $O/r5_01_pytest.log
for r in 1 2 3; do
  for v in "--ramp 4" "--ramp 0"; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 $v > $O/r5_01_cur.json 2> $O/r5_01_cur.err || { tail -20 $O/r5_01_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_01_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['replays'])")" | tee -a $O/r5_01_window.txt
  done
done
timeout -k 10 200 python bench.py --steps 300 --warmup 20 > $O/r5_01_bench300.json 2> $O/r5_01_bench300.err && cat $O/r5_01_bench300.json
