#!/usr/bin/env python3
"""Round 5 diagnosis (docs/CONCURRENCY.md, "the QSC preprocess forward under concurrency"): the graph plans
that run the QSC preprocess forward (csrc/hip/qsc_mfma.hip qsc2_fwd_kernel) next to other kernels produce p1s /
angles that differ, for ~10% of the samples scattered over all workgroups and XCDs (r5_52), from an eager
recompute of the same kernel on the same inputs.  This probe takes the graphs out: it launches the forward on
one stream while a chosen partner kernel runs on another, many times, and counts the samples whose p1s differ
from a serial launch.  A partner that makes results differ shares the CUs with the forward and disturbs it.

    python scripts/probes/probe_qsc_coresident.py [trials]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import quantum_distributed_machine_learning_ris_channel_estimation_amd._native as nat  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops import fc  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda")
    torch.manual_seed(0)
    ctx = DistContext(device=dev)
    tr = FlagshipTrainer(FlagshipConfig(hip_graphs=False, stream_mode="serial", batch=32, data_len=800,
                                        use_quantumnat=True, qsc_grid_bwd=128), ctx)
    tr.step()
    torch.cuda.synchronize()
    h = tr.cstep.hip
    x, flat = tr.gat.xq.clone(), tr.qspace.flat.clone()
    h._fwd_mfma(x, flat, nat.stream_ptr(dev))
    torch.cuda.synchronize()
    ref_p1, ref_ang = h.p1s.clone(), h.angles.clone()
    print(f"QSC forward: B {h.B} grid {h.grid_fwd} x3 {h.fwd_x3} p1s {tuple(h.p1s.shape)}", flush=True)

    bf = torch.bfloat16
    M, N, K = 4608, 2048, 2048
    A, W = torch.randn(M, K, device=dev, dtype=bf), torch.randn(N, K, device=dev, dtype=bf) * 0.02
    dY = torch.randn(M, N, device=dev, dtype=bf)
    Y, dW, dA = torch.empty(M, N, device=dev, dtype=bf), torch.empty(N, K, device=dev), torch.empty(M, K, device=dev, dtype=bf)
    big = torch.empty(64 << 20, device=dev, dtype=torch.uint8)
    big2 = torch.empty_like(big)
    partners = {
        "none": None,
        "copy": lambda: big2.copy_(big),
        "hipblaslt_linear": lambda: F.linear(A, W),
        "hand_fwd": (lambda: fc.gemm_fwd(A, W, out=Y)) if fc.gemm_fwd_ok(M, N, K) else None,
        "hand_wgrad": (lambda: fc.gemm_wgrad(dY, A, out=dW)) if fc.gemm_wgrad_ok(M, N, K) else None,
        "hand_dgrad": (lambda: fc.gemm_dgrad(dY, W, out=dA)) if fc.gemm_dgrad_ok(M, N, K) else None,
        "qsc_fwd_itself": lambda: h._fwd_mfma(x, flat, nat.stream_ptr(dev)),
    }
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for name, fn in partners.items():
        if fn is None and name != "none":
            print(f"{name}: shape not supported, skipped", flush=True)
            continue
        for order in ("partner_first", "qsc_first"):
            bad_trials = bad_samples = 0
            worst = 0.0
            for _ in range(trials):
                h.p1s.zero_()
                torch.cuda.synchronize()
                if order == "qsc_first":
                    with torch.cuda.stream(s1):
                        h._fwd_mfma(x, flat, nat.stream_ptr(dev))
                if fn is not None:
                    with torch.cuda.stream(s2):
                        for _ in range(3):
                            fn()
                if order == "partner_first":
                    with torch.cuda.stream(s1):
                        h._fwd_mfma(x, flat, nat.stream_ptr(dev))
                torch.cuda.synchronize()
                per = (h.p1s - ref_p1).abs().amax(dim=1)
                nb = int((per > 0).sum())
                bad_trials += nb > 0
                bad_samples += nb
                worst = max(worst, float(per.max()), float((h.angles - ref_ang).abs().max()))
            print(f"{name:18s} {order:13s}: {bad_trials}/{trials} trials differ, {bad_samples} samples, worst {worst:.3e}",
                  flush=True)


if __name__ == "__main__":
    main()
