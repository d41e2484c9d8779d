#!/bin/bash
# round-5 GPU call 65: the exact final library (rebuilt after comment-only edits): smoke, the QSC tests and the split-plan tests
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r5_65_smoke.log 2>&1 || { tail -20 $O/r5_65_smoke.log; exit 1; }
tail -1 $O/r5_65_smoke.log
timeout -k 10 600 python -u -m pytest tests/test_qsc_gpu.py tests/test_flagship_gpu.py -m gpu -x -q -k "qsc or library_fc_forward or multistream" --timeout 200 --timeout-method thread > $O/r5_65_pytest.log 2>&1 || { tail -30 $O/r5_65_pytest.log; exit 1; }
tail -1 $O/r5_65_pytest.log
