"""Bit-exactness of the dagq step's capture-order variants against the serial eager step (round-4 coherence
experiment, docs/CONCURRENCY.md).  QDML_QSC_ORDER selects the variant; prints one line per trial.

    python scripts/r4_order_probe.py TRIALS [BATCH]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


def state(tr):
    return [tr.hdce.space.flat, tr.qspace.flat, tr.hopt.m, tr.hopt.v, tr.qopt.m, tr.qopt.v,
            tr.hdce.fc_shadow] + list(tr.hdce.run_mean) + list(tr.hdce.run_var)


def main(trials, batch):
    dev = torch.device("cuda", 0)
    ctx = DistContext(device=dev)
    base = dict(batch=batch, data_len=max(800, 20 * batch), use_quantumnat=True, qsc_grid_bwd=128)
    bad = 0
    t0 = time.time()
    for t in range(trials):
        ref = FlagshipTrainer(FlagshipConfig(hip_graphs=False, stream_mode="serial", **base), ctx)
        dag = FlagshipTrainer(FlagshipConfig(hip_graphs=True, stream_mode="dagq", steps_per_graph=4, **base), ctx)
        dag.capture(preserve=True, k=4)
        first = None
        for rep in range(3):
            for _ in range(4):
                ref.step()
            dag.run(4)
            torch.cuda.synchronize()
            for i, (a, b) in enumerate(zip(state(ref), state(dag))):
                if not torch.equal(a, b):
                    first = (rep, i, float((a.float() - b.float()).abs().max()))
                    break
            if first:
                break
        bad += first is not None
        print(f"trial {t}: {'MISMATCH ' + str(first) if first else 'ok'}", flush=True)
        del ref, dag
    print(f"order={os.environ.get('QDML_QSC_ORDER', 'qsc_first')} batch={batch} mismatches {bad}/{trials} "
          f"({time.time() - t0:.0f}s)", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]) if len(sys.argv) > 2 else 32)
