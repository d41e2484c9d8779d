"""In-step sweep of the HIP conv stack's launch shapes (ops/conv.py ConvStackHIP: spw = samples per wave of the
forward / dgrad, spb_f = samples per workgroup of the fused layer-3/2 backward, spb_r = of the BN backward
reduction, spb_w1 = of the layer-1 weight gradient) on the flagship P128 step, world 1, bench defaults.

    r4_conv_sweep.py [steps] [rounds]

Each variant builds a fresh trainer (one shared HBM dataset), captures, settles and times `steps` steps with
HIP events; variants alternate over `rounds` rounds.  Prints ms/step per variant and round."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops import conv as conv_mod  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train import engine  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)

VARIANTS = {
    "default": {},
    "spw1": {"spw": 1},
    "spw4": {"spw": 4},
    "spb_f4": {"spb_f": 4},
    "spb_f6": {"spb_f": 6},
    "spb_r2": {"spb_r": 2},
    "spb_r8": {"spb_r": 8},
    "spb_w1_2": {"spb_w1": 2},
    "spb_w1_8": {"spb_w1": 8},
}


def build(kw, store, ctx):
    base = conv_mod.ConvStackHIP

    class Patched(base):
        def __init__(self, model, U, B, **k):
            k.update(kw)
            super().__init__(model, U, B, **k)

    engine.ConvStackHIP = Patched
    try:
        return FlagshipTrainer(FlagshipConfig(), ctx, store=store)
    finally:
        engine.ConvStackHIP = base


def timed(tr, steps):
    tr.prepare(steps)
    tr.run(3 * tr._k())
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    tr.run(steps)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ctx = DistContext(device=torch.device("cuda"))
    only = os.environ.get("SWEEP_ONLY")
    names = [n for n in VARIANTS if not only or n in only.split(",")]
    res = {n: [] for n in names}
    store = None
    for r in range(rounds):
        for n in names:
            t0 = time.time()
            tr = build(VARIANTS[n], store, ctx)
            store = tr.store
            tr.run(10)
            ms = timed(tr, steps)
            res[n].append(ms)
            print(f"round {r} {n:10s} {ms:.4f} ms/step  ({time.time() - t0:.1f} s)", flush=True)
            del tr
            torch.cuda.empty_cache()
    for n in names:
        print(f"{n:10s} " + " ".join(f"{v:.4f}" for v in res[n]) + f"   min {min(res[n]):.4f}")


if __name__ == "__main__":
    main()
