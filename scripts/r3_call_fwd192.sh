#!/bin/bash
# Round-3 GPU call: the hand-written FC forward on 192 x 128 tiles (cfg 1: 192 tiles, so ~64 CUs stay free for
# the concurrent QSC branch, as hipBLASLt's 234-tile MT128x160 kernel leaves 22), with the loss epilogue (fwd)
# and with the bias-only epilogue + NMSE pass (fwdplain); same-box step A/B at P128 and P256.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
STEPS="variants" VARIANTS="NONE=0|;QDML_HAND_GEMM=fwd,wgrad,dgrad QDML_GEMM_CFG=1,1,2|;QDML_HAND_GEMM=fwdplain,wgrad,dgrad QDML_GEMM_CFG=1,1,2|;NONE=0|--pilot 256 --qubits 12;QDML_HAND_GEMM=fwd,wgrad,dgrad QDML_GEMM_CFG=1,1,2|--pilot 256 --qubits 12;QDML_HAND_GEMM=fwdplain,wgrad,dgrad QDML_GEMM_CFG=1,1,2|--pilot 256 --qubits 12" bash scripts/gpu_check.sh
