#!/bin/bash
# round-5 GPU call 47: call 46's suite segfaulted (host side, in the graph replay of
# test_multistream_graph_matches_serial_eager[indep+conv-False-3], twice) -- that test alone, then its file alone
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -u -X faulthandler -m pytest "tests/test_flagship_gpu.py::test_multistream_graph_matches_serial_eager" -x -v --timeout 200 --timeout-method thread > $O/r5_47_single.log 2>&1; rc=$?
echo "single rc=$rc"; tail -5 $O/r5_47_single.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -X faulthandler -m pytest tests/test_flagship_gpu.py -x -q --timeout 200 --timeout-method thread > $O/r5_47_file.log 2>&1; rc=$?
echo "file rc=$rc"; tail -5 $O/r5_47_file.log
