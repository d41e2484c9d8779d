#!/bin/bash
# round-5 GPU call 10: stream_mode "indep" (QSC and HDCE chains independent for the whole replay, each with its own
# gather: no cross-queue edge on the HDCE chain): bit-exactness against the serial eager step, then the step A/B
# against dagq, 3 alternating rounds; the P256 step likewise
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_flagship_gpu.py -x -q -k "multistream or bit_exact" --timeout 200 --timeout-method thread > $O/r5_10_pytest.log 2>&1 || { tail -40 $O/r5_10_pytest.log; exit 1; }
tail -2 $O/r5_10_pytest.log
for r in 1 2 3; do
  for v in dagq indep; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 --stream-mode $v > $O/r5_10_cur.json 2> $O/r5_10_cur.err || { tail -20 $O/r5_10_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_10_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['final_losses'])")" | tee -a $O/r5_10_ab.txt
  done
done
for r in 1 2; do
  for v in dagq indep; do
    timeout -k 10 200 python bench.py --pilot 256 --qubits 12 --steps 100 --warmup 10 --stream-mode $v > $O/r5_10_cur.json 2> $O/r5_10_cur.err || { tail -20 $O/r5_10_cur.err; exit 1; }
    echo "round $r [p256 $v] $(python -c "import json; d=json.load(open('$O/r5_10_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'])")" | tee -a $O/r5_10_ab.txt
  done
done
