#!/bin/bash
# round-5 GPU call 8: the MFMA simulators with padded LDS planes (<= 2-way bank conflicts) and packed fp16 splits:
# numerics, isolated kernel times against the VALU kernels, and the P256 / 12-qubit step A/B
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qsim12_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r5_08_pytest.log 2>&1 || { tail -40 $O/r5_08_pytest.log; exit 1; }
tail -2 $O/r5_08_pytest.log
timeout -k 10 300 python scripts/probes/probe_qsim_mfma.py 5 > $O/r5_08_qsim_probe.txt 2>&1; cat $O/r5_08_qsim_probe.txt
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python bench.py --qsim-mfma12 $v --pilot 256 --qubits 12 --steps 100 --warmup 10 > $O/r5_08_cur.json 2> $O/r5_08_cur.err || { tail -20 $O/r5_08_cur.err; exit 1; }
    echo "round $r [p256 q12 mfma12=$v] $(python -c "import json; d=json.load(open('$O/r5_08_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'])")" | tee -a $O/r5_08_p256.txt
  done
done
# the HDCE loss in the FC forward's epilogue (hand "fwd") on the producer-wave 144 x 128 tile vs the plain forward +
# the one-pass NMSE kernel (round 4 measured the epilogue slower on the 4-stage 192 x 128 tile)
for r in 1 2 3; do
  for v in "fwdplain,wgrad,dgrad" "fwd,wgrad,dgrad"; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 --knob hand_gemm=$v > $O/r5_08_cur.json 2> $O/r5_08_cur.err || { tail -20 $O/r5_08_cur.err; exit 1; }
    echo "round $r [$v] $(python -c "import json; d=json.load(open('$O/r5_08_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'], d['config']['fc_forward'], d['final_losses'])")" | tee -a $O/r5_08_fwd_epi.txt
  done
done
