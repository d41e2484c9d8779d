#!/usr/bin/env python3
"""Time the hand-written FC GEMMs (csrc/hip/gemm.hip, every cfg) against hipBLASLt (TunableOp choices when
the shipped file exists) at the flagship shape M=2304, N=2048, K=4096, on uniform random operands.
Rounds interleave the variants in one process (guide §5.4 rule 24); the median and min are printed."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import (  # noqa: E402
    gemm_dgrad, gemm_dgrad_f8, gemm_fwd, gemm_fwd_f8, gemm_nt_f8, gemm_wgrad, gemm_wgrad_f8, transpose_u8)


def timeit(fn, iters=30):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dev = torch.device("cuda")
    M, N, K = 2304, 2048, 4096
    A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    W = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
    b = (torch.rand(N, device=dev) * 2 - 1).bfloat16()
    dY = (torch.rand(M, N, device=dev) * 2 - 1).bfloat16()
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    dW = torch.empty(N, K, device=dev)
    dA = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    fl = 2 * M * N * K
    A8, W8 = A.to(torch.float8_e4m3fn), W.to(torch.float8_e4m3fn)
    deq = torch.ones(2, device=dev)
    one = torch.ones(1, device=dev)
    dY8 = dY.to(torch.float8_e4m3fn)
    Wt8, dYt8, At8 = W8.t().contiguous(), dY8.t().contiguous(), A8.t().contiguous()
    dW8o = torch.empty(N, K, device=dev)
    var = {
        "wgrad_f8_rowmajor": lambda: gemm_wgrad_f8(dY8, A8, one, one, out=dW8o),
        "dgrad_f8_rowmajor": lambda: gemm_dgrad_f8(dY8, W8, one, one, out=dA),
        "dgrad_f8mx_c1": lambda: gemm_nt_f8(dY8, Wt8, one, one, out=dA, cfg=1),
        "dgrad_f8mx_c2": lambda: gemm_nt_f8(dY8, Wt8, one, one, out=dA, cfg=2),
        "wgrad_f8mx_c2": lambda: gemm_nt_f8(dYt8, At8, one, one, out=dW8o, cfg=2),
        "transpose_A8": lambda: transpose_u8(A8, out=At8),
        "transpose_W8": lambda: transpose_u8(W8, out=Wt8),
        "fwd_f8_0": lambda: gemm_fwd_f8(A8, W8, deq, b, out=Y, cfg=0),
        "fwd_f8_mx": lambda: gemm_fwd_f8(A8, W8, deq, b, out=Y, cfg=1),
        "fwd_hipblaslt": lambda: torch.nn.functional.linear(A, W, b),
        "fwd_hand0": lambda: gemm_fwd(A, W, b, out=Y, cfg=0),
        "fwd_hand1": lambda: gemm_fwd(A, W, b, out=Y, cfg=1),
        "fwd_hand2_ks2": lambda: gemm_fwd(A, W, b, out=Y, cfg=2),
        "fwd_hand3_4x1": lambda: gemm_fwd(A, W, b, out=Y, cfg=3),
        "fwd_hand4_2x2": lambda: gemm_fwd(A, W, b, out=Y, cfg=4),
        "fwd_hand5_directA": lambda: gemm_fwd(A, W, b, out=Y, cfg=5),
        "fwd_hand6_b4": lambda: gemm_fwd(A, W, b, out=Y, cfg=6),
        "fwd_hand0_noload": lambda: gemm_fwd(A, W, b, out=Y, cfg=101),
        "fwd_hand0_nomfma": lambda: gemm_fwd(A, W, b, out=Y, cfg=102),
        "wgrad_hipblaslt": lambda: torch.mm(dY.t(), A, out_dtype=torch.float32, out=dW),
        "wgrad_hand0": lambda: gemm_wgrad(dY, A, out=dW, cfg=0),
        "wgrad_hand1": lambda: gemm_wgrad(dY, A, out=dW, cfg=1),
        "wgrad_hand2_ks2": lambda: gemm_wgrad(dY, A, out=dW, cfg=2),
        "wgrad_hand3_2x2": lambda: gemm_wgrad(dY, A, out=dW, cfg=3),
        "wgrad_hand4_b4": lambda: gemm_wgrad(dY, A, out=dW, cfg=4),
        "dgrad_hipblaslt": lambda: torch.mm(dY, W, out=dA),
        "dgrad_hand0": lambda: gemm_dgrad(dY, W, out=dA, cfg=0),
        "dgrad_hand1": lambda: gemm_dgrad(dY, W, out=dA, cfg=1),
        "dgrad_hand2_1x8": lambda: gemm_dgrad(dY, W, out=dA, cfg=2),
        "dgrad_hand3_ks2": lambda: gemm_dgrad(dY, W, out=dA, cfg=3),
        "dgrad_hand4_288": lambda: gemm_dgrad(dY, W, out=dA, cfg=4),
    }
    # cold-cache variants: a 512 MB write evicts L2 and the MALL before the GEMM (the step's FC operands
    # arrive from HBM: the weight shadow was written a whole step earlier); subtract flush_only
    flush = torch.empty(128 << 20, device=dev)
    var["flush_only"] = lambda: flush.zero_()
    var["fwd_hand1_cold"] = lambda: (flush.zero_(), gemm_fwd(A, W, b, out=Y, cfg=1))
    var["wgrad_hand1_cold"] = lambda: (flush.zero_(), gemm_wgrad(dY, A, out=dW, cfg=1))
    var["dgrad_hand2_cold"] = lambda: (flush.zero_(), gemm_dgrad(dY, W, out=dA, cfg=2))
    if os.environ.get("PROBE_ONLY"):
        keep = os.environ["PROBE_ONLY"].split(",")
        var = {k: v for k, v in var.items() if k in keep}
    res = {k: [] for k in var}
    for _ in range(5):
        for k, f in var.items():
            res[k].append(timeit(f))
    for k, v in res.items():
        med = statistics.median(v)
        print(f"{k:18s} median {med:8.2f} us  min {min(v):8.2f} us  {fl / med / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    main()
