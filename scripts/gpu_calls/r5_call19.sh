#!/bin/bash
# round-5 GPU call 19 (run twice: v1 with the slab workgroups after the regular ones, v2 with them first): the HDCE Adam summing the step's gradient slabs itself (KNOBS.adam_slabs: the slab launch off
# the chain) -- optimizer / flagship tests incl. on == off bit for bit, then the step A/B, 3 alternating rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_flagship_gpu.py tests/test_kernels_gpu.py -x -q -k "adam or slab or multistream or bit_exact or optim" --timeout 200 --timeout-method thread > $O/r5_19_pytest.log 2>&1 || { tail -40 $O/r5_19_pytest.log; exit 1; }
tail -1 $O/r5_19_pytest.log
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_19_cur.json 2> $O/r5_19_cur.err || { tail -20 $O/r5_19_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_19_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_19_ab_v2.txt
}
for r in 1 2 3; do
  run "r$r adam_slabs"
  run "r$r slab_launch" --knob adam_slabs=0
done
