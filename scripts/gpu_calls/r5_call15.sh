#!/bin/bash
# round-5 GPU call 15: the FC weight's Adam overlapping the next step's gather + conv forward (fc_adam_next, indep
# plan): bit-exactness tests, then the step A/B against the default, 3 alternating rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_flagship_gpu.py -x -q -k "multistream or bit_exact" --timeout 200 --timeout-method thread > $O/r5_15_pytest.log 2>&1 || { tail -40 $O/r5_15_pytest.log; exit 1; }
tail -1 $O/r5_15_pytest.log
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_15_cur.json 2> $O/r5_15_cur.err || { tail -20 $O/r5_15_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_15_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'], d['config']['fc_adam_next'])")" | tee -a $O/r5_15_ab.txt
}
for r in 1 2 3; do
  run "r$r default"
  run "r$r fc_adam_next" --fc-adam-next
done
