#!/bin/bash
# world-1 RCCL A/B: coalesced-bucket scatter-back as one multi-tensor launch vs one copy per member
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2; do for v in "QDML_BUCKET_FOREACH=1|--dp-graph one" "QDML_BUCKET_FOREACH=0|--dp-graph one" "QDML_BUCKET_FOREACH=1|--dp-graph five" "QDML_BUCKET_FOREACH=0|--dp-graph five"; do
  env QDML_FORCE_DIST=1 ${v%%|*} timeout -k 10 300 python bench.py --steps 300 --warmup 10 --phase-steps 0 ${v#*|} > $OUT/bk.log 2>&1 || { tail -20 $OUT/bk.log; exit 1; }
  echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/bk.log)" | tee -a $OUT/bucket_ab.txt
done; done
