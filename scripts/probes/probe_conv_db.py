#!/usr/bin/env python3
"""Round 6: the conv stack alone (no QSC chain beside it), forward and backward, with and without the
software-pipelined kernels (KNOBS.conv_fwd_db / conv_bwd_db), timed with HIP events over back-to-back iterations.

    python scripts/probes/probe_conv_db.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.conv import ConvStackHIP
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel
    dev = torch.device("cuda")
    U, B = 3, 256
    m = HDCEModel(128, dev, "bf16")
    x1 = torch.randn(U * B, 2 * m.E, m.H, m.W, device=dev)
    dh = torch.randn(U * B * m.E, 32 * m.H * m.W, device=dev).to(torch.bfloat16)
    for rnd in range(2):
        for fdb, bdb, spb in ((False, False, 5), (True, False, 5), (False, True, 10), (False, True, 9), (False, False, 10)):
            KNOBS.conv_fwd_db, KNOBS.conv_bwd_db, KNOBS.conv_spb_db = fdb, bdb, spb
            cs = ConvStackHIP(m, U, B, spb_f=spb)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            for i in range(iters):
                if i == iters // 2:
                    ev[0].record()
                cs.forward(x1, True)
            ev[1].record()
            for i in range(iters):
                if i == iters // 2:
                    ev[2].record()
                cs.backward(dh)
            ev[3].record()
            torch.cuda.synchronize()
            n = iters - iters // 2
            print(f"round {rnd} fwd_db={int(fdb)} bwd_db={int(bdb)} spb={spb}: forward stack "
                  f"{ev[0].elapsed_time(ev[1]) / n * 1e3:.1f} us, backward stack {ev[2].elapsed_time(ev[3]) / n * 1e3:.1f} us",
                  flush=True)
            del cs


if __name__ == "__main__":
    main()
