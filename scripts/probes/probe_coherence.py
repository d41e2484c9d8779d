"""Cross-queue coherence probe: is a consumer kernel that a HIP graph runs on another hardware queue, right after
a cross-queue edge from its producer, guaranteed to see the producer's writes?  (docs/CONCURRENCY.md: the
QSC-chain stale read; csrc/hip/runtime.hip coh_* kernels.)

Per step, captured k steps per graph: produce(buf) on main -> fork -> consume(buf) on a side stream while main
runs a busy kernel (so the executor maps the branch to its own queue) -> join -> tick(step counter).  buf is
1 MiB, so the consumer's previous-step lines stay in its XCDs' L2.  Every variant replays R graphs and reports
elements that did not hold the step's value (bad) and those that held the previous step's value (stale).

    probe_coherence.py [replays] [steps per graph]
"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat  # noqa: E402

_p, _i = ctypes.c_void_p, ctypes.c_int
N = 1 << 18          # ints (1 MiB)
GRID = 512           # consumer / producer workgroups (spread over all 8 XCDs)


def fns():
    lib = nat.hip_lib()
    return (nat.fn(lib, "qd_coh_produce", [_p, _i, _p, _i, _p]), nat.fn(lib, "qd_coh_consume", [_p, _i, _p, _p, _i, _i, _p]),
            nat.fn(lib, "qd_coh_tick", [_p, _p]), nat.fn(lib, "qd_coh_busy", [_p, _i, _i, _i, _p]))


def variant(place, mode, replays, k):
    produce, consume, tick, busy = fns()
    dev = torch.device("cuda")
    buf = torch.zeros(N, dtype=torch.int32, device=dev)
    ctr = torch.ones(1, dtype=torch.int32, device=dev)
    errs = torch.zeros(2, dtype=torch.int32, device=dev)
    junk = torch.rand(1 << 20, device=dev)
    side = torch.cuda.Stream()

    def step():
        st = nat.stream_ptr()
        nat.check(produce(nat.ptr(buf), N, nat.ptr(ctr), GRID, st), "produce")
        if place == "cross":
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                nat.check(consume(nat.ptr(buf), N, nat.ptr(ctr), nat.ptr(errs), mode, GRID, nat.stream_ptr()),
                          "consume")
            nat.check(busy(nat.ptr(junk), junk.numel(), 64, 256, st), "busy")
            main.wait_stream(side)
        else:
            nat.check(consume(nat.ptr(buf), N, nat.ptr(ctr), nat.ptr(errs), mode, GRID, st), "consume")
        nat.check(tick(nat.ptr(ctr), st), "tick")

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(k):
            step()
    errs.zero_()
    c0 = int(ctr.item())
    t0 = time.perf_counter()
    for _ in range(replays):
        g.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = int(ctr.item()) - c0
    e = errs.tolist()
    print(f"{place:5s} mode {mode}  steps {steps:6d}  bad {e[0]:10d}  stale {e[1]:10d}  "
          f"({dt / max(1, steps) * 1e6:.1f} us/step)", flush=True)
    return e


def main():
    replays = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    for place, mode in (("same", 0), ("cross", 0), ("cross", 1), ("cross", 2), ("cross", 0)):
        variant(place, mode, replays, k)


if __name__ == "__main__":
    main()
