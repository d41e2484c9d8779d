#!/bin/bash
# A/B of the training step between the in-tree library ("new") and lib_ab/libqdml_hip_base.so ("base"), alternating
# on one box: ab_lib.sh TAG ROUNDS [bench args...]  ->  gpurun_out/TAG_ab.txt
cd "$(dirname "$0")/.." || exit 1
R=$(pwd); O=$R/gpurun_out; L=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd/lib
TAG=$1; N=$2; shift 2
cp $L/libqdml_hip.so $R/lib_ab/libqdml_hip_new.so
for r in $(seq 1 $N); do
  for v in new base; do
    cp $R/lib_ab/libqdml_hip_$v.so $L/libqdml_hip.so
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 "$@" > $O/${TAG}_bench_$v.json 2>$O/${TAG}_bench_$v.err || { cp $R/lib_ab/libqdml_hip_new.so $L/libqdml_hip.so; exit 1; }
    echo "round $r $v $(python -c "import json; print(json.load(open('$O/${TAG}_bench_$v.json'))['ms_per_step'])")" >> $O/${TAG}_ab.txt
  done
done
cp $R/lib_ab/libqdml_hip_new.so $L/libqdml_hip.so
