#!/bin/bash
# Build the A side of an A/B run: the kernel source FILE (under csrc/hip) as of git revision REV, linked with
# the tree's current objects of every other source, into lib/libqdml_hip_base.so.  A GPU call script swaps it
# in place of lib/libqdml_hip.so for the A runs and back (scripts/gpu_calls/r5_call11.sh).
# Usage: scripts/build_ab_lib.sh REV conv.hip   (after the in-tree build)
set -eo pipefail
REV=$1; F=$2
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/quantum_distributed_machine_learning_ris_channel_estimation_amd
T=$(mktemp -d)
git -C "$R" show "$REV:quantum_distributed_machine_learning_ris_channel_estimation_amd/csrc/hip/$F" > "$T/$F"
EXTRA=$(python -c "import sys; sys.path.insert(0, '$R'); from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as n; print(' '.join(n.PER_FILE_FLAGS.get('$F', [])))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=fast -Wno-unused-result $EXTRA \
  -I "$P/csrc/hip" -c "$T/$F" -o "$T/$F.o"
OBJS=$(ls "$P"/lib/obj/*.o | grep -v "/$F.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$P/lib/libqdml_hip_base.so" $OBJS "$T/$F.o"
rm -rf "$T"
echo "built $P/lib/libqdml_hip_base.so ($F at $REV)"
