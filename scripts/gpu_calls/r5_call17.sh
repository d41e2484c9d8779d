#!/bin/bash
# round-5 GPU call 17: the indep step with the HDCE chain captured on a high-priority stream (hdce_priority), the
# FC Adam overlapping the next conv forward on capped grids (fc_adam_next 256 / 512), and the QSC chain's grids (the
# preprocess forward's cap KNOBS.qsc_fwd_cap 256 -> 576, the backward's qsc_grid_bwd 256 -> 128 / 512): tests + 3
# alternating rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_flagship_gpu.py -x -q -k "multistream or bit_exact" --timeout 200 --timeout-method thread > $O/r5_17_pytest.log 2>&1 || { tail -40 $O/r5_17_pytest.log; exit 1; }
tail -1 $O/r5_17_pytest.log
run() {   # label, bench args...
  local lab=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/r5_17_cur.json 2> $O/r5_17_cur.err || { tail -20 $O/r5_17_cur.err; exit 1; }
  echo "[$lab] $(python -c "import json; d=json.load(open('$O/r5_17_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_17_ab.txt
}
for r in 1 2 3; do
  run "r$r default"
  run "r$r hdce_priority" --hdce-priority
  run "r$r fc_adam_next256" --fc-adam-next 256
  run "r$r fc_adam_next512" --fc-adam-next 512
  run "r$r fwdcap576" --knob qsc_fwd_cap=576
  run "r$r bwd512" --qsc-grid-bwd 512
  run "r$r bwd128" --qsc-grid-bwd 128
done
