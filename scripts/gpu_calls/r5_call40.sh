#!/bin/bash
# round-5 GPU call 40: the split-forward + fused-loss QSC mismatch under LDS poisoning (every launch preceded by an
# LDS fill of the whole chip: NaN pattern, then a zero pattern) -- does the QSC preprocess forward read LDS it did not
# write?
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
R=$(pwd); O=$R/gpurun_out
for pat in FFFFFFFF 00000000 3F800000; do
  echo "== poison $pat" >> $O/r5_40_poison.txt
  PROBE_LDS_POISON=$pat timeout -k 10 200 python -u scripts/probes/probe_split_fused.py fwd fcnext 1 >> $O/r5_40_poison.txt 2>&1 || { tail -20 $O/r5_40_poison.txt; exit 1; }
done
grep "== poison\|^step\|p1s\|angles" $O/r5_40_poison.txt
