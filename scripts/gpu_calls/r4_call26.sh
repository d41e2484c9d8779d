#!/bin/bash
# round-4 GPU call: Adam access-pattern variants, cold (after a 512 MB flush)
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python scripts/probes/r4_adam_probe.py > $O/r4_26_adam_probe.txt 2>&1 || exit 1
