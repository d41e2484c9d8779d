#!/usr/bin/env python3
"""QSC step alone (no HDCE chain beside it) for kernel traces: the P128 backward on bf16x3 MFMAs
(qsc2_bwd3_kernel) and on f32 MFMAs (QDML_QSC_BWD=f32 / --f32)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--f32", action="store_true")
    a = ap.parse_args()
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import QSC_P128
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.optim import FlatParamSpace
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.qsc import QSCStepHIP
    dev = torch.device("cuda")
    B = 2304
    m = QSC_P128(n_qubits=8, use_quantumnat=True, use_gradient_pruning=False).to(dev)
    sp = FlatParamSpace(list(m.named_parameters()), dev)
    step = QSCStepHIP(m, sp, B, n_groups=9)
    step.bwd_x3 = step.bwd_x3 and not a.f32
    x = torch.randn(B, 2, 16, 8, device=dev)
    y = torch.randint(0, 3, (B,), device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for i in range(a.iters):
        if i == a.iters // 2:
            ev[0].record()
        step(x, y)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"bf16x3={step.bwd_x3} QSC step {ev[0].elapsed_time(ev[1]) / (a.iters - a.iters // 2) * 1e3:.1f} us")


if __name__ == "__main__":
    main()
