#!/bin/bash
# round-5 GPU call 61: the other headline configurations on the final tree (P256 / 12 qubits, its b1024 config, 16 qubits +
# fp8, the forced DP plan at world 1, bench.py with no arguments)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python bench.py --pilot 256 --qubits 12 --steps 100 --warmup 10 > $O/r5_61_bench_p256.json 2>$O/r5_61_bench_p256.err || exit 1
timeout -k 10 300 python bench.py --pilot 256 --qubits 12 --batch 1024 --steps 30 --warmup 5 > $O/r5_61_bench_p256_b1024.json 2>$O/r5_61_bench_p256_b1024.err || exit 1
timeout -k 10 300 python bench.py --qubits 16 --dtype fp8 --steps 20 --warmup 3 > $O/r5_61_bench_q16.json 2>$O/r5_61_bench_q16.err || exit 1
QDML_FORCE_DIST=1 timeout -k 10 400 python bench.py --steps 200 --warmup 20 --select-steps 30 > $O/r5_61_bench_forced.json 2>$O/r5_61_bench_forced.err || exit 1
timeout -k 10 120 python bench.py > $O/r5_61_bench_default_args.json 2>$O/r5_61_bench_default_args.err || exit 1
for f in p256 p256_b1024 q16 forced default_args; do python -c "import json; d=json.load(open('$O/r5_61_bench_$f.json')); print('$f', d['ms_per_step'], d['value'], d['final_losses'])"; done
