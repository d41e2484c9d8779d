# dbg_bisect over build variants: VARIANTS="none -DQD_VLOAD=1 -DQD_SLEEP_US=3" CASES="dagi:2 qsc:1" TRIALS=30
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
for v in ${VARIANTS:-none}; do
  f=$v; [ "$v" = none ] && f=""
  QDML_HIPCC_EXTRA="$f" timeout -k 10 300 python -c "from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as n; n.build_hip(force=True, verbose=False)" || exit 1
  for c in ${CASES:-dagi:2}; do
    timeout -k 10 400 python -u scripts/dbg_bisect.py ${c%%:*} ${c##*:} 6 ${TRIALS:-30} > gpurun_out/var_${v//[-=]/}_${c/:/}.log 2>&1 || exit $?
    echo "$v $(grep SUMMARY gpurun_out/var_${v//[-=]/}_${c/:/}.log)"
  done
done
