#!/usr/bin/env python3
"""Round 6: the streamed 16-qubit simulator (csrc/hip/qsim_stream.hip) alone at the flagship batch -- forward with
kept states + adjoint backward, n = 16, L = 3, 2,304 samples in 9 weight groups (QuantumNAT) -- timed with HIP events
over back-to-back iterations (also the program the PMC passes profile).

    python scripts/probes/probe_qstream.py [iters]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    lib = nat.hip_lib()
    _p, _i = ctypes.c_void_p, ctypes.c_int
    dev = torch.device("cuda")
    n, L, B, G = 16, 3, 256, 9
    BB = B * G
    torch.manual_seed(0)
    x = torch.rand(BB, n, device=dev) * 3.0 - 1.5
    w = torch.rand(G, L, n, 2, device=dev) * 6.28
    gE = torch.randn(BB, n, device=dev)
    st = nat.stream_ptr(dev)
    rows = nat.fn(lib, "qd_qsim_stream_rows", [_i])(BB)
    ws = torch.empty(nat.fn(lib, "qd_qsim_stream_workspace", [_i, _i, _i, _i], ctypes.c_longlong)(n, BB, L, 1),
                     dtype=torch.uint8, device=dev)
    ps = torch.empty(nat.fn(lib, "qd_qsim_stream_save_bytes", [_i, _i, _i], ctypes.c_longlong)(n, BB, L),
                     dtype=torch.uint8, device=dev)
    sf = nat.fn(lib, "qd_qsim_stream_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
    sb = nat.fn(lib, "qd_qsim_stream_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
    E, dx = torch.empty(BB, n, device=dev), torch.empty(BB, n, device=dev)
    slab = torch.empty(rows, 2 * n * L, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for i in range(iters):
        if i == iters // 2:
            ev[0].record()
        nat.check(sf(nat.ptr(x), nat.ptr(w), nat.ptr(E), BB, n, L, B, nat.ptr(ws), nat.ptr(ps), st), "stream fwd")
        if i == iters // 2:
            ev[1].record()
        nat.check(sb(nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), BB, n, L, B, nat.ptr(ws),
                     nat.ptr(ps), st), "stream bwd")
        if i == iters // 2:
            ev[2].record()
    torch.cuda.synchronize()
    print(f"n=16 L=3 B={BB}: forward {ev[0].elapsed_time(ev[1]):.3f} ms, backward {ev[1].elapsed_time(ev[2]):.3f} ms, "
          f"finite {bool(torch.isfinite(dx).all())}", flush=True)


if __name__ == "__main__":
    main()
