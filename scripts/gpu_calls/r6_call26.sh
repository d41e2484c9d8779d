#!/bin/bash
# round-6 GPU call 26: the reverse pass B gathering lambda with all 16 loads in flight before its LDS scatter (layer
# 0's pass ran at 2.8 TB/s with 4 at a time): kernel tests + LDS poison, config 5 twice, the step's kernel stats
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_26
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_lds_poison_gpu.py -x -q --timeout 240 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
B q16_1 python bench.py --steps 30 --warmup 5 --qubits 16 --gradient-pruning --dtype fp8
B q16_2 python bench.py --steps 30 --warmup 5 --qubits 16 --gradient-pruning --dtype fp8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --qubits 16 --gradient-pruning --dtype fp8 > $O/${P}_prof.log 2>&1 || { tail -5 $O/${P}_prof.log; exit 1; }
db=$(find $O/${P}_prof -name '*.db' | head -1)
python scripts/prof_summary.py $db --tail 0.6 > $O/${P}_q16_kernel_stats.md 2>&1; head -16 $O/${P}_q16_kernel_stats.md
rm -rf $O/${P}_prof
