#!/usr/bin/env python3
"""Per-phase cycle breakdown of the HDCE conv kernel (layer-2 forward and the bf16 data-gradient
pass) from in-kernel s_memtime stamps (diagnostic build path qd_conv_stamped)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.conv import ConvStackHIP
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel
    dev = torch.device("cuda")
    U, B, E = 3, 256, 3
    m = HDCEModel(128, dev, "bf16")
    x1 = torch.randn(U * B, 2 * E, m.H, m.W, device=dev)
    dh = torch.randn(U * B * E, 32 * m.H * m.W, device=dev).to(torch.bfloat16)
    f = nat.fn(nat.hip_lib(), "qd_conv_stamped", [ctypes.c_int] + [ctypes.c_void_p] * 6 + [ctypes.c_int] * 5
               + [ctypes.c_void_p] * 2)
    names = ["weights+params", "first sample staged", "first sample MFMA+epilogue", "remaining samples", "stats tail"]
    out = {}
    for spw, dg in ((2, 0), (2, 1), (1, 0), (1, 1)):
        cs = ConvStackHIP(m, U, B, spw=spw)
        for _ in range(3):
            cs.forward(x1, True)
            cs.backward(dh)
        torch.cuda.synchronize()
        grid = U * cs.chunks * E
        st = torch.zeros(grid * 4 * 8, dtype=torch.int64, device=dev)
        for _ in range(3):
            if dg == 0:
                args = (nat.ptr(cs.z[0]), None, nat.ptr(cs.st[0]), nat.ptr(cs.wpk[1]), nat.ptr(cs.z[1]),
                        nat.ptr(cs.stats[1]))
            else:
                args = (nat.ptr(dh), nat.ptr(cs.z[2]), nat.ptr(cs.st[2]), nat.ptr(cs.wpk_t[2]), nat.ptr(cs.dx[1]),
                        None)
            nat.check(f(dg, *args, cs.N, E, B, cs.chunks, cs.spw, nat.ptr(st), nat.stream_ptr(dev)), "stamped")
        torch.cuda.synchronize()
        t = st.view(grid * 4, 8).cpu().double()
        d = {nm: float((t[:, i + 1] - t[:, i]).median()) for i, nm in enumerate(names)}
        d["wave_lifetime_median"] = float((t[:, 5] - t[:, 0]).median())
        d["wave_lifetime_max"] = float((t[:, 5] - t[:, 0]).max())
        out[("dgrad" if dg else "forward_layer2") + f"_spw{spw}"] = d
    # isolated wall time of the whole stack (3 forward launches + BN tail; backward launches)
    cs = ConvStackHIP(m, U, B)
    for _ in range(5):
        cs.forward(x1, True)
        cs.backward(dh)
    for nm, fn in (("forward", lambda: cs.forward(x1, True)), ("backward", lambda: cs.backward(dh))):
        ts = []
        for _ in range(30):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        ts.sort()
        out[f"isolated_{nm}_us"] = {"median": ts[len(ts) // 2], "min": ts[0]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
