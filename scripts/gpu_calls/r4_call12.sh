#!/bin/bash
# round-4 GPU call: full GPU suite on the join-before-update plan, bench + step timeline, QSC-gate probe (P256 / P128),
# 16-qubit bench repeat
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r4_12_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/r4_12_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/r4_12_bench.json 2>$O/r4_12_bench.err || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_step -o run -- python $R/bench.py --steps 100 --warmup 20 > $O/tl_step.log 2>&1) || exit 1
python scripts/prof_timeline.py $O/tl_step/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r4_12_step_timeline.md
python scripts/prof_summary.py $O/tl_step/run_kernel_trace.csv --tail 0.6 > $O/r4_12_step_kernel_stats.md; rm -rf $O/tl_step
timeout -k 10 400 python scripts/probes/r4_qsc_gate_probe.py 256 12 100 2 > $O/r4_12_qsc_gate_p256.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/probes/r4_qsc_gate_probe.py 128 8 300 2 > $O/r4_12_qsc_gate_p128.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --qubits 16 --dtype fp8 --steps 20 --warmup 3 > $O/r4_12_bench_q16.json 2>$O/r4_12_bench_q16.err || exit 1
QDML_FORCE_DIST=1 timeout -k 10 400 python bench.py --steps 200 --warmup 20 --select-steps 30 > $O/r4_12_bench_forced.json 2>$O/r4_12_bench_forced.err || exit 1
timeout -k 10 120 python scripts/probes/probe_coherence.py 300 10 > $O/r4_12_coherence.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/probes/stamp_conv.py > $O/r4_12_stamp_conv.txt 2>&1 || exit 1
timeout -k 10 180 python scripts/probes/r4_adam_probe.py > $O/r4_12_adam_probe.txt 2>&1 || exit 1
timeout -k 10 180 python scripts/probes/probe_qsc_determinism.py 40 > $O/r4_12_qsc_determinism.txt 2>&1 || exit 1
