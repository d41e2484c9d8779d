#!/bin/bash
# round-6 GPU call 46: the streamed simulator's backward run chunk by chunk (QDML_QSTREAM_CHUNK samples: all layers
# per chunk, the chunk-sized lambda buffers kept in the Infinity Cache between passes): kernel tests at the default
# and at chunk 2; the probe at chunk 0 / 64 / 128 / 256; config 5 at 0 / 128 / 256, 2 rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out; P=r6_46
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread -k "stream or qsim" > $O/${P}_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest.log
tail -2 $O/${P}_pytest.log
[ $rc -eq 0 ] || exit 1
QDML_QSTREAM_CHUNK=2 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread -k "stream or qsim" > $O/${P}_pytest_chunk2.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/${P}_pytest_chunk2.log
tail -2 $O/${P}_pytest_chunk2.log
[ $rc -eq 0 ] || exit 1
for c in 0 64 128 256; do
  timeout -k 10 200 env QDML_QSTREAM_CHUNK=$c python -u scripts/probes/probe_qstream.py 6 2>&1 | grep n=16 | sed "s/^/chunk=$c /" | tee -a $O/${P}_probe.txt
done
B() { n=$1; shift; timeout -k 10 400 "$@" > $O/${P}_$n.json 2>$O/${P}_$n.err || { tail -5 $O/${P}_$n.err; exit 1; }; python -c "import json; d=json.load(open('$O/${P}_$n.json')); print('$n', d['ms_per_step'], d['replays'][:3], d['step_spread']['median_ms'], d['steps_trained'], d['final_losses'])" | tee -a $O/${P}_ab.txt; }
for r in 1 2; do
  for c in 0 128 256; do
    B c${c}_$r env QDML_QSTREAM_CHUNK=$c python bench.py --steps 30 --warmup 5 --qubits 16 --gradient-pruning --dtype fp8
  done
done
