#!/bin/bash
# round-4 GPU call: P256 / 12-qubit QSC fork placement (the simulator backward crowds the NMSE pass out), 2 rounds;
# the forced world-1 bench's stdout (one JSON line, the RCCL banner on stderr)
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
PILOT=256 QUBITS=12 ROUNDS=2 PLAN=shipped,fork_conv2,fork_conv3 timeout -k 10 500 python scripts/probes/r4_plan_probe.py 100 > $O/r4_24_plans_p256.txt 2>&1 || exit 1
QDML_FORCE_DIST=1 timeout -k 10 400 python bench.py --steps 100 --warmup 20 --select-steps 30 > $O/r4_24_bench_forced.json 2>$O/r4_24_bench_forced.err || exit 1
