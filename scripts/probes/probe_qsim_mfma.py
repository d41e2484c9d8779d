#!/usr/bin/env python3
"""Isolated timing of the quantum simulators at the flagship batch (2304 samples, 3 layers, 9 QuantumNAT groups):
12 qubits -- csrc/hip/qsim12_mfma.hip (MFMA mode products) vs qsim_big.hip (VALU); 8 qubits -- the adjoint on the
MFMA (qd_qsim_mfma8_bwd) vs qsim.hip's register kernel.  Median over rounds interleaving the variants.

    python scripts/probes/probe_qsim_mfma.py [rounds]"""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat  # noqa: E402

_p, _i = ctypes.c_void_p, ctypes.c_int


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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    lib = nat.hip_lib()
    dev = torch.device("cuda")
    B, L, G = 2304, 3, 9
    st = nat.stream_ptr(dev)
    var = {}
    for n in (12, 8):
        x = torch.rand(B, n, device=dev) * 3
        w = torch.rand(G, L, n, 2, device=dev) * 6.28
        gE = torch.randn(B, n, device=dev) / B
        E, dx = torch.empty(B, n, device=dev), torch.empty(B, n, device=dev)
        ps = torch.empty(B * (8 << n), dtype=torch.uint8, device=dev)
        wg = B // G
        if n == 12:
            rows = nat.fn(lib, "qd_qsim_big_grid", [_i])(B)
            slab = torch.empty(rows, 2 * n * L, device=dev)
            ws = torch.empty(nat.fn(lib, "qd_qsim_mfma12_workspace", [_i, _i], ctypes.c_longlong)(G, L),
                             dtype=torch.uint8, device=dev)
            ff = nat.fn(lib, "qd_qsim_mfma12_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
            fb = nat.fn(lib, "qd_qsim_mfma12_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
            vf = nat.fn(lib, "qd_qsim_big_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
            vb = nat.fn(lib, "qd_qsim_big_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
            var["q12_fwd_mfma"] = lambda ff=ff, x=x, w=w, E=E, ws=ws, ps=ps, wg=wg: ff(
                nat.ptr(x), nat.ptr(w), nat.ptr(E), B, 12, L, wg, nat.ptr(ws), nat.ptr(ps), st)
            var["q12_bwd_mfma"] = lambda fb=fb, x=x, w=w, gE=gE, dx=dx, slab=slab, ws=ws, ps=ps, wg=wg: fb(
                nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, 12, L, wg, nat.ptr(ws), nat.ptr(ps),
                st)
            var["q12_fwd_valu"] = lambda vf=vf, x=x, w=w, E=E, ps=ps, wg=wg: vf(
                nat.ptr(x), nat.ptr(w), nat.ptr(E), B, 12, L, wg, None, nat.ptr(ps), st)
            var["q12_bwd_valu"] = lambda vb=vb, x=x, w=w, gE=gE, dx=dx, slab=slab, ps=ps, wg=wg: vb(
                nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, 12, L, wg, None, nat.ptr(ps), st)
            # (the MFMA backward reads the MFMA forward's psave layout, the VALU backward its own: keep each pair's
            # state consistent by running the forward first in each timing)
            fwm, bwm, fwv, bwv = var["q12_fwd_mfma"], var.pop("q12_bwd_mfma"), var["q12_fwd_valu"], var.pop("q12_bwd_valu")
            var["q12_fb_mfma"] = lambda fwm=fwm, bwm=bwm: (fwm(), bwm())
            var["q12_fb_valu"] = lambda fwv=fwv, bwv=bwv: (fwv(), bwv())
        else:
            rows = nat.fn(lib, "qd_qsim_bwd_grid", [_i, _i])(n, B)
            slab = torch.empty(rows, 2 * n * L, device=dev)
            ws = torch.empty(nat.fn(lib, "qd_qsim_mfma8_workspace", [_i, _i], ctypes.c_longlong)(G, L),
                             dtype=torch.uint8, device=dev)
            nat.check(nat.fn(lib, "qd_qsim_fwd_save", [_p, _p, _p, _i, _i, _i, _i, _p, _p])(
                nat.ptr(x), nat.ptr(w), nat.ptr(E), B, n, L, wg, nat.ptr(ps), st), "fwd_save")
            mb = nat.fn(lib, "qd_qsim_mfma8_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
            rb = nat.fn(lib, "qd_qsim_bwd_saved", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p])
            var["q8_bwd_mfma"] = lambda mb=mb, x=x, w=w, gE=gE, dx=dx, slab=slab, ws=ws, ps=ps, wg=wg: mb(
                nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, 8, L, wg, nat.ptr(ws), nat.ptr(ps),
                st)
            var["q8_bwd_reg"] = lambda rb=rb, x=x, w=w, gE=gE, dx=dx, slab=slab, ps=ps, wg=wg: rb(
                nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, 8, L, wg, nat.ptr(ps), st)
    ts = {k: [] for k in var}
    for _ in range(rounds):
        for k, fn in var.items():
            ts[k].append(timeit(fn))
    for k, v in ts.items():
        print(f"{k:14s} median {statistics.median(v):9.2f} us  min {min(v):9.2f} us", flush=True)


if __name__ == "__main__":
    main()
