#!/bin/bash
# round-6 GPU call 18 (second run: compile-time samples per workgroup, all their loads in flight at P128): the conv
# forward on conv3x3_split_kernel -- the conv tests, the forward-stack probe (P128 / P256, sps sweep), the bench
# alternating base / split sps 5 / split sps 4, 2 rounds, and a kernel-stats profile of the probe
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_18
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py -x -q -s --timeout 240 --timeout-method thread > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -3 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/probes/probe_conv_split.py 60 > $O/${P}_probe.txt 2>&1 || { tail -5 $O/${P}_probe.txt; exit 1; }
cat $O/${P}_probe.txt
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2; do
  B base_$r python bench.py --steps 200 --warmup 10
  B split5_$r python bench.py --steps 200 --warmup 10 --knob conv_fwd_split=1 --knob conv_sps=5
  B split4_$r python bench.py --steps 200 --warmup 10 --knob conv_fwd_split=1 --knob conv_sps=4
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${P}_prof -o run -- python3 $R/scripts/probes/probe_conv_split.py 40 > $O/${P}_prof.log 2>&1 || { tail -5 $O/${P}_prof.log; exit 1; }
db=$(find $O/${P}_prof -name '*.db' | head -1)
python scripts/prof_summary.py $db --tail 1.0 --top 30 > $O/${P}_probe_kernel_stats.md 2>&1; head -30 $O/${P}_probe_kernel_stats.md
rm -rf $O/${P}_prof
