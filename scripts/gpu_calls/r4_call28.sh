#!/bin/bash
# conv VALU diet: in-kernel phase stamps and isolated stack times, new library vs the previous one
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; L=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd/lib
cp $L/libqdml_hip.so $R/lib_ab/libqdml_hip_new.so
for v in new base new base; do
  cp $R/lib_ab/libqdml_hip_$v.so $L/libqdml_hip.so
  echo "== $v" >> $O/r4_28_stamp_conv.txt
  timeout -k 10 120 python scripts/probes/stamp_conv.py >> $O/r4_28_stamp_conv.txt 2>&1 || exit 1
done
cp $R/lib_ab/libqdml_hip_new.so $L/libqdml_hip.so
