#!/bin/bash
# round-5 GPU call 50: is call 46's segfault the code?  The full GPU suite with the library built from the reverted
# gemm.hip (cfg 11 + the batched loss-epilogue loads, commit 92b0831; scripts/build_ab_lib.sh -> libqdml_hip_base.so)
# swapped in.  (test_gemm_gpu's cfg-11 cases are not in this tree: it runs the final tree's tests.)
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
L=quantum_distributed_machine_learning_ris_channel_estimation_amd/lib
cp $L/libqdml_hip.so $O/final.so && cp $L/libqdml_hip_base.so $L/libqdml_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5_50_pytest.log 2>&1; rc=$?
cp $O/final.so $L/libqdml_hip.so && rm -f $O/final.so
echo "pytest rc=$rc"; tail -3 $O/r5_50_pytest.log
