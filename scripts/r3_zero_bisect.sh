#!/bin/bash
# Round-3 bisection of the gloo-on-one-GPU QSC mismatch: (a) the same plan twice (run-to-run determinism of
# each plan), (b) the QSC branch on the main stream (stream_mode serial) vs forked (dagq).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
one() {   # label env...
  local label=$1; shift
  rm -f /tmp/zb.*
  env "$@" timeout -k 10 240 python -c "
import sys; sys.path.insert(0, '.')
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch import launch
sys.exit(launch([sys.executable, 'tests/dist_scripts/zero_vs_allreduce.py', '/tmp/zb', 'cuda'], nproc=2,
                extra_env={'OMP_NUM_THREADS': '2', 'QDML_DIST_BACKEND': 'gloo'}))" > $OUT/zb.log 2>&1 || { tail -20 $OUT/zb.log; exit 1; }
  echo "$label: $(cat /tmp/zb.0)" | tee -a $OUT/r3_zero_bisect.txt
}
for r in $(seq 1 ${ROUNDS:-3}); do
  one "r$r serial zero-vs-allreduce" QDML_STREAM_MODE=serial || exit 1
  one "r$r dagq allreduce-vs-allreduce" QDML_ZV_PLANS=allreduce,allreduce || exit 1
  one "r$r dagq zero-vs-zero" QDML_ZV_PLANS=zero,zero || exit 1
done
