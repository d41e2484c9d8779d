#!/bin/bash
# round-4 GPU call: shipped vs QSC fork after conv 1 (whole HDCE chain on one queue), 3 alternating rounds
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
ROUNDS=3 PLAN=shipped,fork_conv1 timeout -k 10 400 python scripts/probes/r4_plan_probe.py 400 > $O/r4_19_plans.txt 2>&1 || exit 1
