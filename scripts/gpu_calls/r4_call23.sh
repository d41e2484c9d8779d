#!/bin/bash
# round-4 GPU call: forward tile configs in the step after the 4-stage default (6: 192x128 4-stage, 0: 144x128 4-stage
# on 256 tiles, 2: 144x128 split-K 2)
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
VARIANTS="N=0|;N=1|--gemm-cfg 0,1,2;N=2|--gemm-cfg 2,1,2" bash scripts/gpu_calls/r4_ab.sh $O/r4_23_ab.txt || exit 1
