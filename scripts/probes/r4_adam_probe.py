"""Isolated timing of the flat Adam kernel over the FC_P128 parameter count (8.39 M) vs plain HBM streams of the
same byte count (torch copies), to see how far the update is from the achievable read+write bandwidth."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.optim import (  # noqa: E402
    FlatParamSpace, make_optimizer)


def timeit(fn, iters=20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dev = torch.device("cuda")
    n = 2048 * 4096 + 2048
    p = torch.nn.Parameter(torch.randn(n, device=dev) * 0.02)
    space = FlatParamSpace([("w", p)], dev)
    opt = make_optimizer(space, "adam", 1e-3)
    sh = opt.attach_shadow(0, n - n % 4)
    space.grad.normal_()
    flush = torch.empty(128 << 20, device=dev)
    src = torch.empty(n * 4, device=dev)        # 4 fp32 streams read ...
    dst = torch.empty(n * 3, device=dev)        # ... 3 written (+ the bf16 shadow ~ 0.5 more)
    def adam_grid(g):
        def f():
            opt.max_grid[0] = g
            opt.step()
        return f

    var = {
        "adam": lambda: opt.step(),
        "copy_r4w3": lambda: dst.copy_(src[:n * 3]),
        "read4": lambda: src.sum(),
        "flush_then_adam": lambda: (flush.zero_(), opt.step()),
        "flush_only": lambda: flush.zero_(),
    }
    # launch sizes of the update (cold, as in the step: after a 512 MB flush), grid-stride over 8.4 M params
    for g in (1024, 4096, 8192):
        var[f"flush_then_adam_grid{g}"] = (lambda f: lambda: (flush.zero_(), f()))(adam_grid(g))
    var["flush_then_adam_grid2048"] = (lambda f: lambda: (flush.zero_(), f()))(adam_grid(2048))
    # access-pattern variants of the same update (csrc/hip/optim.hip qd_adam_probe), cold
    import ctypes
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    vp = ctypes.c_void_p
    fprobe = nat.fn(nat.hip_lib(), "qd_adam_probe", [ctypes.c_int, vp, vp, vp, vp, ctypes.c_long, vp, vp,
                                                     ctypes.c_float, ctypes.c_float, ctypes.c_float, vp,
                                                     ctypes.c_int, vp])
    shadow = torch.empty(n, device=dev, dtype=torch.bfloat16)

    def probe(variant, grid):
        def f():
            flush.zero_()
            nat.check(fprobe(variant, nat.ptr(space.flat), nat.ptr(space.grad), nat.ptr(opt.m), nat.ptr(opt.v), n,
                             nat.ptr(opt.lr_t), nat.ptr(opt.step_t), 0.9, 0.999, 1e-8, nat.ptr(shadow), grid,
                             nat.stream_ptr()), "adam_probe")
        return f
    names = {0: "nt_nt_u1", 1: "nt_nt_u2", 2: "ld_nt_u1", 3: "nt_st_u1", 4: "plain_u1", 5: "nt_nt_u4", 6: "plain_u2"}
    for vnum, nm in names.items():
        for grid in (2048, 8192):
            var[f"flush_then_probe_{nm}_g{grid}"] = probe(vnum, grid)
    bytes_adam = n * (4 * 4 + 3 * 4 + 2)
    res = {k: [] for k in var}
    for _ in range(5):
        for k, f in var.items():
            res[k].append(timeit(f))
    for k, v in res.items():
        med = statistics.median(v)
        print(f"{k:16s} median {med:8.2f} us  min {min(v):8.2f} us   adam-bytes rate {bytes_adam / med / 1e6:6.2f} TB/s")


if __name__ == "__main__":
    main()
