#!/usr/bin/env python3
"""Conv-stack backward alone (no QSC chain beside it): ConvStackHIP.backward in a loop, for rocprofv3
kernel traces / PMC passes of the fused conv3x3_bwd_kernel vs the side-by-side wd kernel.

    python scripts/probes/probe_conv_bwd.py [--fused 0|1] [--spb-f S] [--iters N] [--pilot 128|256]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pilot", type=int, default=128)
    ap.add_argument("--spb-f", type=int, default=5)
    ap.add_argument("--fused", type=int, default=1)
    a = ap.parse_args()
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.conv import ConvStackHIP
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel
    dev = torch.device("cuda")
    U, B = 3, 256
    m = HDCEModel(a.pilot, dev, "bf16")
    cs = ConvStackHIP(m, U, B, bwd_fused=bool(a.fused), spb_f=a.spb_f)
    x1 = torch.randn(U * B, 2 * m.E, m.H, m.W, device=dev)
    dh = torch.randn(U * B * m.E, 32 * m.H * m.W, device=dev).to(torch.bfloat16)
    cs.forward(x1, True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for i in range(a.iters):
        if i == a.iters // 2:
            ev[0].record()
        cs.backward(dh)
    ev[1].record()
    torch.cuda.synchronize()
    n = a.iters - a.iters // 2
    print(f"fused={cs.bwd_fused} spb_f={a.spb_f} backward {ev[0].elapsed_time(ev[1]) / n * 1e3:.1f} us/iter")


if __name__ == "__main__":
    main()
