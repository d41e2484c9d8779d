#!/bin/bash
# Round-3 diagnosis of the gloo-on-one-GPU ZeRO-vs-all-reduce mismatch (docs/CONCURRENCY.md): the same
# 2-rank comparison with and without a host sync after every gloo work.wait(), alternating, N rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-3}); do
  for hs in 0 1; do
    rm -f /tmp/zd.*
    QDML_GLOO_HOST_SYNC=$hs timeout -k 10 240 python -c "
import sys; sys.path.insert(0, '.')
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch import launch
sys.exit(launch([sys.executable, 'tests/dist_scripts/zero_vs_allreduce.py', '/tmp/zd', 'cuda'], nproc=2,
                extra_env={'OMP_NUM_THREADS': '2', 'QDML_DIST_BACKEND': 'gloo'}))" > $OUT/zd.log 2>&1 || { tail -20 $OUT/zd.log; exit 1; }
    echo "round $r host_sync=$hs: $(cat /tmp/zd.0)" | tee -a $OUT/r3_zero_diag.txt
  done
done
