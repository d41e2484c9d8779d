#!/bin/bash
# round-4 GPU call: HDCE Adam launch size in the step (2048 shipped vs 1024 / 1536 workgroups), 3 rounds
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
ROUNDS=3 PLAN=shipped,adam1024,adam1536 timeout -k 10 500 python scripts/probes/r4_plan_probe.py 400 > $O/r4_20_plans.txt 2>&1 || exit 1
