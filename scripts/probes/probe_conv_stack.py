"""Isolated timing of the conv stack's training forward: the per-layer launches (3 conv + BN tail) against the
persistent launch (conv.hip conv_fwd_stack_kernel), each captured in a HIP graph and replayed; also each alone
beside a concurrent load on a second stream (a QSC step of the flagship) to see how the persistent kernel's
barriers fare when other kernels hold CUs.

    python scripts/probes/probe_conv_stack.py [reps]
    QDML_STACK_STAMPS=1 python scripts/probes/probe_conv_stack.py     # per-phase stamps of the persistent kernel
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.conv import ConvStackHIP  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda")
    U, B = 3, 256
    torch.manual_seed(0)
    m = HDCEModel(128, dev, "bf16")
    x1 = m.pack_input(torch.randn(3, U, B, 2, m.H, m.W, device=dev)).contiguous()
    res = {}
    for stack in (False, True):
        KNOBS.conv_stack = stack
        conv = ConvStackHIP(m, U, B)
        assert conv.stack == stack
        conv.forward(x1, training=True)
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            conv.forward(x1, training=True)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=st):
                for _ in range(10):
                    conv.forward(x1, training=True)
        torch.cuda.synchronize()
        t = timed(g.replay, max(1, reps // 10)) / 10
        res["stack" if stack else "per-layer"] = t
        if stack:
            assert not conv.stack_error()
    for k, v in res.items():
        print(f"{k:10s} forward {v:8.2f} us")


def stamps(reps=20):
    """Per-workgroup phase stamps of the persistent forward (qd_conv_fwd_stack_stamped): body / barrier cycles."""
    import ctypes
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    dev = torch.device("cuda")
    U, B = 3, 256
    torch.manual_seed(0)
    m = HDCEModel(128, dev, "bf16")
    x1 = m.pack_input(torch.randn(3, U, B, 2, m.H, m.W, device=dev)).contiguous()
    KNOBS.conv_stack = True
    conv = ConvStackHIP(m, U, B)
    conv.pack_weights(nat.stream_ptr(dev))
    grid = U * conv.chunks * conv.E
    buf = torch.zeros(grid * 8, dtype=torch.int64, device=dev)
    f = nat.fn(nat.hip_lib(), "qd_conv_fwd_stack_stamped", [ctypes.c_void_p] * 2 + [ctypes.c_int] * 5
               + [ctypes.c_void_p] * 2)
    a = conv.stack_args(x1)
    rows = []
    for _ in range(reps):
        nat.check(f(ctypes.byref(a), nat.ptr(conv.stack_sync), conv.N, conv.E, conv.B, conv.chunks, conv.spw,
                    nat.ptr(buf), nat.stream_ptr(dev)), "stack stamped")
        torch.cuda.synchronize()
        rows.append(buf.view(grid, 8).cpu().double())
    assert not conv.stack_error()
    names = ["L1 body", "barrier 1", "L2 body", "barrier 2", "L3 body", "barrier 3", "tail"]
    t = torch.stack(rows)                       # (reps, grid, 8)
    d = t[..., 1:] - t[..., :-1]
    print(f"{'phase':10s} {'median':>8s} {'p90':>8s} {'max':>8s}  (cycles, over {reps} runs x {grid} workgroups)")
    for k, n in enumerate(names):
        v = d[..., k].flatten()
        print(f"{n:10s} {v.median():8.0f} {v.quantile(0.9):8.0f} {v.max():8.0f}")
    start = t[..., 0] - t[..., 0].min(dim=1, keepdim=True).values
    life = t[..., 7] - t[..., 0]
    print(f"start spread: median {start.median():.0f} max {start.max():.0f}; workgroup lifetime median "
          f"{life.median():.0f} max {life.max():.0f}; kernel span median "
          f"{(t[..., 7].max(1).values - t[..., 0].min(1).values).median():.0f}")


if __name__ == "__main__":
    if os.environ.get("QDML_STACK_STAMPS"):   # per-phase stamps of the persistent kernel
        stamps()
    else:
        main()
