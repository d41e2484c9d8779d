#!/bin/bash
# round-4 GPU call: conv kernel phase stamps, Adam launch-size sweep
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 120 python scripts/probes/stamp_conv.py > $O/r4_13_stamp_conv.txt 2>&1 || exit 1
timeout -k 10 180 python scripts/probes/r4_adam_probe.py > $O/r4_13_adam_probe.txt 2>&1 || exit 1
timeout -k 10 180 python scripts/probes/probe_qsc_determinism.py 40 > $O/r4_13_qsc_determinism.txt 2>&1 || exit 1
