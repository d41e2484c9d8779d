set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stream or qsim_big" > gpurun_out/t_stream.log 2>&1; rc=$?; tail -3 gpurun_out/t_stream.log; [ $rc -ne 0 ] && exit $rc
for q in 16 15 14 13; do for s in 1 0; do QDML_QSIM_STREAM=$s timeout -k 10 300 python bench.py --steps 6 --warmup 2 --steps-per-graph 1 --qubits $q > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }; echo "q$q stream=$s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b.log)"; done; done
