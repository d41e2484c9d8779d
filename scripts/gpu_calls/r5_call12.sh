#!/bin/bash
# round-5 GPU call 12: (1) the BN tail for groups that are not a multiple of 8 samples (test-time BN re-estimation);
# (2) the persistent conv forward isolated vs the per-layer launches, and its in-step timeline (it measured 12 %
# slower in the step, r5_11_ab.txt); (3) FIG1 with the HDCE weight average + BN adaptation, K = 10 and 30;
# (4) P256 dagq vs indep
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_infer_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r5_12_pytest.log 2>&1 || { tail -40 $O/r5_12_pytest.log; exit 1; }
tail -1 $O/r5_12_pytest.log
timeout -k 10 120 python scripts/probes/probe_conv_stack.py 400 > $O/r5_12_conv_stack_probe.txt 2>&1 || { cat $O/r5_12_conv_stack_probe.txt; exit 1; }
cat $O/r5_12_conv_stack_probe.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stack -o run -- python $R/bench.py --steps 40 --warmup 10 --knob conv_stack=1 > $O/prof_stack.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_stack/run_kernel_trace.csv --tail 0.6 > $O/r5_12_stack_kernel_stats.md
python scripts/prof_timeline.py $O/prof_stack/run_kernel_trace.csv --marker "conv_fwd_stack_kernel" --back 3 > $O/r5_12_stack_timeline.md; rm -rf $O/prof_stack
head -30 $O/r5_12_stack_timeline.md
for K in 10 30; do
  timeout -k 10 900 python -u scripts/train_eval.py --epochs 100 --qubits 6 --out $O/r5_fig1_swa$K --workspace /tmp/ws_swa$K \
    --bn-adapt --swa-epochs $K > $O/r5_12_fig1_swa$K.log 2>&1 || { tail -30 $O/r5_12_fig1_swa$K.log; exit 1; }
  tail -1 $O/r5_12_fig1_swa$K.log
done
for r in 1 2; do
  for v in dagq indep; do
    timeout -k 10 200 python bench.py --pilot 256 --qubits 12 --steps 100 --warmup 10 --stream-mode $v > $O/r5_12_cur.json 2> $O/r5_12_cur.err || { tail -20 $O/r5_12_cur.err; exit 1; }
    echo "round $r [p256 $v] $(python -c "import json; d=json.load(open('$O/r5_12_cur.json')); print(d['ms_per_step'], d['step_spread']['median_ms'])")" | tee -a $O/r5_12_p256_ab.txt
  done
done
