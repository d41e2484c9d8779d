# streamed simulator + e4m3 GEMM: GPU tests, 16/14-qubit and fp8 bench, 16-qubit kernel profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_gpu.py -k "stream or qsim_big or f8" > gpurun_out/t_stream.log 2>&1; rc=$?; tail -5 gpurun_out/t_stream.log; [ $rc -ne 0 ] && exit $rc
for q in "--qubits 16 --dtype fp8" "--qubits 16" "--qubits 14" "--dtype fp8 --steps-per-graph 5 --steps 50" "--steps-per-graph 5 --steps 50"; do timeout -k 10 300 python bench.py --steps 6 --warmup 2 --steps-per-graph 1 $q > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }; echo "$q $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b.log)"; done
[ -n "${PROF:-}" ] && bash scripts/prof_q16.sh
exit 0
