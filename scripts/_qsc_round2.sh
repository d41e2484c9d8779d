R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 200 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_qsc_gpu.py -m gpu > $O/pt.log 2>&1; rc=$?
grep -E "angles|passed|failed|Error" $O/pt.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python scripts/stamp_qsc.py > $O/sq.log 2>&1 || exit 1
bash scripts/_probe_qsc.sh || exit 1
cd $R
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/b$i.log 2>&1 || exit 1
  QDML_QSC_F32=1 timeout -k 10 120 python bench.py --steps 300 --warmup 10 > $O/c$i.log 2>&1 || exit 1
done
