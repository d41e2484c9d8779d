"""Isolated timing of the conv stack's training forward: the per-layer launches (3 conv + BN tail) against the
persistent launch (conv.hip conv_fwd_stack_kernel), each captured in a HIP graph and replayed; also each alone
beside a concurrent load on a second stream (a QSC step of the flagship) to see how the persistent kernel's
barriers fare when other kernels hold CUs.

    python scripts/probe_conv_stack.py [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

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


if __name__ == "__main__":
    main()
