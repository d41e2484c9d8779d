set -o pipefail
cd $GRAFT_REPO_ROOT; OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT
for cfg in "q16:--qubits 16 --dtype fp8 --steps 6 --warmup 2 --steps-per-graph 1" "p256q12:--pilot 256 --qubits 12 --steps 30 --warmup 5" "q16bf16:--qubits 16 --steps 6 --warmup 2 --steps-per-graph 1"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python bench.py $args > $OUT/bench_$name.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$name.log
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$name -o run -- python $GRAFT_REPO_ROOT/bench.py $args > $OUT/prof_$name.log 2>&1) || exit 1
  python scripts/prof_summary.py $OUT/prof_$name/run_kernel_trace.csv --tail 0.5 > $OUT/prof_${name}_summary.md || exit 1
  head -14 $OUT/prof_${name}_summary.md
  rm -rf $OUT/prof_$name
done
