# DP plan at world 1 over a real 1-rank RCCL process group: QSC placement (dp_qsc_phase) x plan
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-"2 zero" "3 zero" "1 zero" "2 zero" "3 zero" "1 zero" "3 allreduce" "2 allreduce"}; do set -- $v
  QDML_FORCE_DIST=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --dp-qsc-phase $1 --dp-plan $2 > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
  echo "phase=$1 plan=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b.log) $(grep -o '"dist_backend": "[a-z]*"' gpurun_out/b.log) $(grep -o '"phases_ms": {[^}]*}' gpurun_out/b.log)"
done
