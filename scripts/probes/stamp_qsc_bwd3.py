#!/usr/bin/env python3
"""Per-phase cycle breakdown of the bf16x3 QSC backward (qsc2_bwd3_kernel) from in-kernel s_memtime
stamps (diagnostic entry qd_qsc2_bwd3_stamped): medians over the waves of the first sample's phases."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import QSC_P128
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.optim import FlatParamSpace
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.qsc import QSCStepHIP
    dev = torch.device("cuda")
    B, n = 2304, 8
    m = QSC_P128(n_qubits=n, use_quantumnat=False, use_gradient_pruning=False).to(dev)
    sp = FlatParamSpace(list(m.named_parameters()), dev)
    step = QSCStepHIP(m, sp, B, n_groups=9)
    x = torch.randn(B, 2, 16, 8, device=dev)
    y = torch.randint(0, 3, (B,), device=dev)
    for _ in range(3):
        step(x, y)
    torch.cuda.synchronize()
    lib = nat.hip_lib()
    gb = step.grid_bwd
    st = torch.zeros(gb * 4 * 12, dtype=torch.int64, device=dev)
    f = nat.fn(lib, "qd_qsc2_bwd3_stamped", [ctypes.c_void_p] * 12 + [ctypes.c_int] * 5 + [ctypes.c_void_p] * 2)
    for _ in range(3):
        nat.check(f(nat.ptr(x), nat.ptr(sp.flat), step.offs, nat.ptr(step.angles), nat.ptr(step.dang),
                    nat.ptr(step.dpre), nat.ptr(step.preslab), nat.ptr(step.p2), *step._saved(), nat.ptr(step.qslab),
                    step.qrows, 2 * n * step.L, B, n, gb, nat.ptr(st), nat.stream_ptr(dev)), "bwd3 stamped")
    torch.cuda.synchronize()
    t = st.view(gb * 4, 12).cpu().double()
    names = ["prologue", "staging", "linear + pool-2 bwd", "conv2 wgrad", "conv2 dgrad", "pool-1 bwd",
             "conv1 wgrad", "other samples", "reduction + slab"]
    out = {nm: float((t[:, i + 1] - t[:, i]).median()) for i, nm in enumerate(names)}
    out["wave_lifetime_median"] = float((t[:, 9] - t[:, 0]).median())
    out["wave_lifetime_max"] = float((t[:, 9] - t[:, 0]).max())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
