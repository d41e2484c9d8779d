#!/bin/bash
# round-5 GPU call 51: the full GPU suite + smoke with the per-test teardown (synchronise, collect the test's graphs)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r5_51_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/r5_51_pytest.log
tail -3 $O/r5_51_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r5_51_smoke.log 2>&1 || { tail -20 $O/r5_51_smoke.log; exit 1; }
tail -1 $O/r5_51_smoke.log
