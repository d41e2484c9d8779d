#!/bin/bash
# bench.py's auto DP graph choice on one GPU (QDML_FORCE_DIST=1 one-rank RCCL group, plain and under
# torchrun): the capture pre-flight, the one-graph all-reduce plan, per-phase timing on the 5-graph plan.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
QDML_FORCE_DIST=1 timeout -k 10 300 python bench.py --steps 300 --warmup 10 > $OUT/auto_plain.log 2>&1 || { tail -30 $OUT/auto_plain.log; exit 1; }
tail -2 $OUT/auto_plain.log
QDML_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 300 --warmup 10 > $OUT/auto_torchrun.log 2>&1 || { tail -30 $OUT/auto_torchrun.log; exit 1; }
tail -2 $OUT/auto_torchrun.log
