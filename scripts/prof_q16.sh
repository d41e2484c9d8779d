# 16-qubit flagship config: bench + rocprofv3 kernel summary (streamed simulator passes)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT
args=${ARGS:-"--qubits 16 --dtype fp8 --steps 6 --warmup 2 --steps-per-graph 1"}
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_q16 -o run -- python $GRAFT_REPO_ROOT/bench.py $args > $OUT/prof_q16.log 2>&1) || exit 1
python scripts/prof_summary.py $OUT/prof_q16/run_kernel_trace.csv --tail 0.5 > $OUT/prof_q16_summary.md || exit 1
head -24 $OUT/prof_q16_summary.md
rm -rf $OUT/prof_q16
