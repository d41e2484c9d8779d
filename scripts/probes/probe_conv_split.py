#!/usr/bin/env python3
"""Round 6: the conv stack's training forward alone (no QSC chain beside it) on conv3x3_kernel (spw samples per
wave) against conv3x3_split_kernel (each sample split over a workgroup's 4 waves, sps samples per workgroup), timed
with HIP events over back-to-back iterations; P128 and P256.

    python scripts/probes/probe_conv_split.py [iters] [pilots, e.g. 128,256] [samples per workgroup, e.g. 0,4,5,6 (0: the
    conv3x3_kernel baseline)]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    pilots = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [128, 256]
    cfgs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 4, 5, 6]
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.conv import ConvStackHIP
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel
    dev = torch.device("cuda")
    for pilot in pilots:
        B = 256
        U = 3
        m = HDCEModel(pilot, dev, "bf16")
        x1 = torch.randn(U * B, 2 * m.E, m.H, m.W, device=dev)
        for rnd in range(2):
            for sps in cfgs:
                split = sps > 0
                KNOBS.conv_fwd_split, KNOBS.conv_sps = split, max(sps, 1)
                cs = ConvStackHIP(m, U, B)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                for i in range(iters):
                    if i == iters // 2:
                        ev[0].record()
                    cs.forward(x1, True)
                ev[1].record()
                torch.cuda.synchronize()
                n = iters - iters // 2
                name = f"split sps={sps}" if split else "conv3x3_kernel"
                print(f"P{pilot} round {rnd} {name}: forward stack {ev[0].elapsed_time(ev[1]) / n * 1e3:.1f} us",
                      flush=True)
                del cs
    KNOBS.conv_fwd_split = False


if __name__ == "__main__":
    main()
