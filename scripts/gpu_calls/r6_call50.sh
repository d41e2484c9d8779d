#!/bin/bash
# round-6 GPU call 50: the one-tile reverse pass A's launch shape -- bricks per workgroup 4 / 2 / 1
# (QDML_QSTREAM_BPB) at the shipped occupancy bound 3, and bound 4 (lib_base: -DQD_STREAM_A1T_OCC=4, 128 VGPRs with
# spills) -- the probe alone, 2 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_50
mkdir -p $O
BASE=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd/lib_base
for r in 1 2; do
  for b in 4 2 1; do
    timeout -k 10 200 env QDML_QSTREAM_BPB=$b python -u scripts/probes/probe_qstream.py 6 2>&1 | grep n=16 | sed "s/^/occ3 bpb$b  /" | tee -a $O/${P}_probe.txt || exit 1
  done
  timeout -k 10 200 env QDML_LIB_DIR=$BASE python -u scripts/probes/probe_qstream.py 6 2>&1 | grep n=16 | sed "s/^/occ4 bpb4  /" | tee -a $O/${P}_probe.txt || exit 1
done
