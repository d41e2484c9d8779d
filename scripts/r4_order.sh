#!/bin/bash
# round-4 capture-order / coherence experiment (docs/CONCURRENCY.md): bit-exactness + step time per variant
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/r4_02_order.txt
: > $O
for v in qsc_first hdce_first own_gather; do
  QDML_QSC_ORDER=$v timeout -k 10 150 python scripts/r4_order_probe.py ${TRIALS:-10} >> $O 2>&1 || exit $?
  QDML_QSC_ORDER=$v timeout -k 10 120 python bench.py --steps 300 --warmup 20 >> $O 2>/dev/null || exit $?
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 QDML_QSC_ORDER=hdce_first timeout -k 10 150 python scripts/r4_order_probe.py ${TRIALS:-10} >> $O 2>&1 || exit $?
