#!/bin/bash
# GPU-box validation: build, smoke, pytest -m gpu, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a timeout/abort/segfault (rc >= 124) ends the script.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-"build smoke pytest bench prof"}
run() {
  local name=$1; shift
  local t0=$(date +%s)
  timeout -k 10 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s" | tee -a "$OUT/summary.txt"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    build) run build 600 python __graft_entry__.py build ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    pytest) run pytest 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ;;
    bench) run bench 600 python bench.py --steps ${BENCH_STEPS:-50} --warmup 10 ;;
    bench_eager) run bench_eager 600 python bench.py --steps 20 --warmup 5 --no-graphs ;;
    bench_p256) run bench_p256 600 python bench.py --steps 20 --warmup 5 --pilot 256 --qubits 12 ;;
    bench_q16) run bench_q16 600 python bench.py --steps 10 --warmup 3 --qubits 16 ;;
    bench_fp8) run bench_fp8 600 python bench.py --steps 50 --warmup 10 --dtype fp8 ;;
    bench_c5) run bench_c5 600 python bench.py --steps 10 --warmup 3 --qubits 16 --dtype fp8 ;;
    train) run train 1200 python scripts/train_eval.py --epochs ${EPOCHS:-100} --qubits 6 --qml-qubits 4,8 --out "$OUT/train" ;;
    pmc) for pc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do n=${pc%% *}; (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $pc --output-format csv -d "$OUT/pmc_$n" -o run -- python "$ROOT/bench.py" --steps 10 --warmup 2 --steps-per-graph 1 > "$OUT/pmc_$n.log" 2>&1) || { echo "pmc $pc failed"; tail -5 "$OUT/pmc_$n.log"; exit 1; }; done; python scripts/pmc_summary.py "$OUT"/pmc_* > "$OUT/pmc_summary.md"; rm -rf "$OUT"/pmc_*/ ;;
    variants) IFS=';' read -ra VS <<< "${VARIANTS:-NONE=0|}"; for r in 1 2; do for v in "${VS[@]}"; do env ${v%%|*} timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-300} --warmup 10 ${v#*|} > $OUT/cmp.log 2>&1 || exit 1; echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/cmp.log)" | tee -a $OUT/variants.txt; done; done ;;
    poison) run poison 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_lds_poison_gpu.py -m gpu ;;
    pytest_fl) run pytest_fl 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flagship_gpu.py -m gpu ;;
    bench_split) run bench_split 600 python bench.py --steps 50 --warmup 10 --split-graphs ;;
    prof) (cd /tmp && export TMPDIR=/tmp && run prof 600 rocprofv3 --kernel-trace ${PROF_EXTRA:-} --stats --output-format csv -d "$OUT/prof" -o run -- python "$ROOT/bench.py" --steps 100 --warmup 5 ${BENCH_EXTRA:-}) && python scripts/prof_summary.py "$OUT/prof/run_kernel_trace.csv" --tail 0.6 > "$OUT/prof_summary.md" && python scripts/prof_timeline.py "$OUT/prof/run_kernel_trace.csv" --marker "conv3x3_kernel<2," > "$OUT/prof_timeline.md" ;;
    prof_fp8) (cd /tmp && export TMPDIR=/tmp && run prof_fp8 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_fp8" -o run -- python "$ROOT/bench.py" --steps 100 --warmup 5 --dtype fp8 --steps-per-graph 1) && python scripts/prof_summary.py "$OUT/prof_fp8/run_kernel_trace.csv" --tail 0.6 > "$OUT/prof_fp8_summary.md" && python scripts/prof_timeline.py "$OUT/prof_fp8/run_kernel_trace.csv" > "$OUT/prof_fp8_timeline.md" ;;
    stamp) run stamp 300 python scripts/probes/stamp_qsc.py ;;
    stamp_conv) run stamp_conv 300 python scripts/probes/stamp_conv.py ;;
    tune) run tune 900 python scripts/tune_kernels.py --what ${TUNE_WHAT:-qsc,conv} ;;
    fp8probe) run fp8probe 300 python scripts/probes/probe_fp8.py ;;
    fcprobe) run fcprobe 300 python scripts/probes/probe_fc_gemm.py ;;
    gemmprobe) run gemmprobe 300 python scripts/probes/probe_gemm.py ;;
    gemmtest) run gemmtest 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -m gpu ;;
    nmseprobe) run nmseprobe 300 python scripts/probes/probe_nmse.py ;;
    diag) run diag 900 python scripts/probes/diag_hdce.py --epochs ${DIAG_EPOCHS:-20} ;;
    gensweep) run gensweep 1500 python scripts/gen_sweep.py --epochs ${SWEEP_EPOCHS:-30} --sc-epochs 8 ;;
  esac
done
# (extra profiles) prof_cfg: PROF_NAME / PROF_ARGS select the bench configuration
if [[ " $STEPS " == *" prof_cfg "* ]]; then
  (cd /tmp && export TMPDIR=/tmp && run prof_${PROF_NAME:-cfg} 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${PROF_NAME:-cfg}" -o run -- python "$ROOT/bench.py" ${PROF_ARGS:-}) && python scripts/prof_summary.py "$OUT/prof_${PROF_NAME:-cfg}/run_kernel_trace.csv" --tail 0.6 > "$OUT/prof_${PROF_NAME:-cfg}_summary.md" && python scripts/prof_timeline.py "$OUT/prof_${PROF_NAME:-cfg}/run_kernel_trace.csv" --back 3 > "$OUT/prof_${PROF_NAME:-cfg}_timeline.md"
fi
