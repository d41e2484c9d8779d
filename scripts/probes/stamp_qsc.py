#!/usr/bin/env python3
"""Per-phase cycle breakdown of the MFMA QSC forward kernel from in-kernel s_memtime stamps
(diagnostic build path qd_qsc2_fwd_stamped).  Prints medians / p90 per phase and the wave
start-time spread (how many 'rounds' of waves the launch needed)."""
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
    waves = nat.fn(lib, "qd_qsc2_waves", [ctypes.c_int, ctypes.c_int])(8, 0)
    grid = step.grid_fwd
    st = torch.zeros(grid * waves * 12, dtype=torch.int64, device=dev)
    f = nat.fn(lib, "qd_qsc2_fwd_stamped", [ctypes.c_void_p] * 8 + [ctypes.c_int] * 5 + [ctypes.c_void_p] * 2)
    for _ in range(3):
        nat.check(f(nat.ptr(x), nat.ptr(sp.flat), step.offs, nat.ptr(step.angles), nat.ptr(step.p2), *step._saved(), B, n,
                    16, 8, grid,
                    nat.ptr(st), nat.stream_ptr(dev)), "stamped")
    torch.cuda.synchronize()
    t = st.view(grid * waves, 12).cpu().double()
    names = ["stage weights", "input tile", "conv1+pool1", "conv2 (MFMA)", "pool2+linear", "rest of samples"]
    out = {}
    for i, nm in enumerate(names):
        d = t[:, i + 1] - t[:, i]
        out[nm] = {"median_cycles": float(d.median()), "p90_cycles": float(d.quantile(0.9))}
    start = t[:, 0] - t[:, 0].min()
    end = t[:, 6] - t[:, 0].min()
    out["wave_start_spread_cycles"] = {"p50": float(start.median()), "p90": float(start.quantile(0.9)),
                                       "max": float(start.max())}
    out["kernel_span_cycles"] = float(end.max())
    out["wave_lifetime_median_cycles"] = float((t[:, 6] - t[:, 0]).median())
    # backward
    wb = nat.fn(lib, "qd_qsc2_waves", [ctypes.c_int, ctypes.c_int])(8, 1)
    gb = step.grid_bwd
    sb = torch.zeros(gb * wb * 12, dtype=torch.int64, device=dev)
    fb = nat.fn(lib, "qd_qsc2_bwd_stamped", [ctypes.c_void_p] * 12 + [ctypes.c_int] * 7 + [ctypes.c_void_p] * 2)
    nat.check(fb(nat.ptr(x), nat.ptr(sp.flat), step.offs, nat.ptr(step.angles), nat.ptr(step.dang), nat.ptr(step.dpre),
                 nat.ptr(step.preslab), nat.ptr(step.p2), *step._saved(), nat.ptr(step.qslab), step.qrows,
                 2 * n * step.L, B, n, 16, 8, gb, nat.ptr(sb),
                 nat.stream_ptr(dev)), "bwd stamped")
    torch.cuda.synchronize()
    tb = sb.view(gb * wb, 12).cpu().double()
    bn = ["stage weights", "saved state -> LDS", "linear + pool2 bwd", "conv2 wgrad (MFMA)", "conv2 dgrad (MFMA)",
          "pool1 bwd (saved argmax)", "conv1 wgrad (MFMA)", "rest of samples + tail"]
    out["backward"] = {nm: float((tb[:, i + 1] - tb[:, i]).median()) for i, nm in enumerate(bn)}
    out["backward"]["wave_lifetime_median_cycles"] = float((tb[:, 8] - tb[:, 0]).median())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
