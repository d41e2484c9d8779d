#!/bin/bash
# round-5 GPU call 9: isolated simulator kernel times (12-qubit MFMA vs VALU, 8-qubit adjoint MFMA vs register) and
# the P256 / 12-qubit step timeline on the current MFMA kernels
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python scripts/probes/probe_qsim_mfma.py 5 > $O/r5_09_qsim_probe.txt 2>&1; cat $O/r5_09_qsim_probe.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p256 -o run -- python $R/bench.py --pilot 256 --qubits 12 --steps 40 --warmup 10 > $O/prof_p256.log 2>&1) || exit 1
python scripts/prof_summary.py $O/prof_p256/run_kernel_trace.csv --tail 0.6 > $O/r5_09_p256_kernel_stats.md
python scripts/prof_timeline.py $O/prof_p256/run_kernel_trace.csv --marker "conv3x3_kernel<2," --back 5 > $O/r5_09_p256_timeline.md; rm -rf $O/prof_p256
cat $O/r5_09_p256_timeline.md
