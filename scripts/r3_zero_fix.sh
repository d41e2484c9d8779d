#!/bin/bash
# Round-3: the gloo-on-one-GPU DP plan run-to-run check (allreduce plan twice) and the ZeRO-vs-all-reduce
# comparison, N rounds, with the simulator's coherent input loads (QD_QSIM_COHERENT_IN, the shipped build).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-4}); do
  for plans in allreduce,allreduce allreduce,zero; do
    rm -f /tmp/zf.*
    QDML_ZV_PLANS=$plans timeout -k 10 240 python -c "
import sys; sys.path.insert(0, '.')
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch import launch
sys.exit(launch([sys.executable, 'tests/dist_scripts/zero_vs_allreduce.py', '/tmp/zf', 'cuda'], nproc=2,
                extra_env={'OMP_NUM_THREADS': '2', 'QDML_DIST_BACKEND': 'gloo'}))" > $OUT/zf.log 2>&1 || { tail -20 $OUT/zf.log; exit 1; }
    echo "r$r $plans: $(cat /tmp/zf.0)" | tee -a $OUT/r3_zero_fix.txt
  done
done
