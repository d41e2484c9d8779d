#!/usr/bin/env python3
"""Where does the driver's short timing window (--steps 20) lose time against --steps 300?  Runs the bench's
world-1 flagship exactly like bench.py (warm-up, capture, settle), then times K steps three ways: host wall
(what bench.py reports), HIP events around the whole window, and HIP events around every graph replay."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lead = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    ctx = DistContext(device=torch.device("cuda", 0))
    tr = FlagshipTrainer(FlagshipConfig(steps_per_graph=5, lead_in=lead), ctx)
    tr.run(5)
    for rnd in range(3):
        tr.prepare(K)
        tr.run(25)
        torch.cuda.synchronize()
        reps = tr._reps(K)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(reps) + 1)]
        t0 = time.perf_counter()
        ev[0].record()
        for i, kk in enumerate(reps):
            tr._replay(kk, fence=i == len(reps) - 1)
            ev[i + 1].record()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        per = [ev[i].elapsed_time(ev[i + 1]) for i in range(len(reps))]
        gpu = ev[0].elapsed_time(ev[-1])
        print(f"K={K} lead={lead} round {rnd}: wall {wall * 1e3 / K:.4f} ms/step, events {gpu / K:.4f} ms/step, "
              f"host enqueue {th * 1e3:.3f} ms; per replay (steps: ms) "
              + " ".join(f"{kk}:{p:.3f}" for kk, p in zip(reps, per)), flush=True)


if __name__ == "__main__":
    main()
