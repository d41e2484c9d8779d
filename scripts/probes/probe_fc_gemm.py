#!/usr/bin/env python3
"""Time the three FC_P128 GEMMs of the flagship step (M = 2304 rows, N = 2048, K = 4096) in the
formulations PyTorch can hand to hipBLASLt / rocBLAS, to pick the fastest per GEMM."""
import json

import torch


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dev = torch.device("cuda")
    M, N, K = 2304, 2048, 4096
    A = torch.randn(M, K, device=dev).bfloat16()
    W = torch.randn(N, K, device=dev).bfloat16() * 0.02
    b = torch.randn(N, device=dev).bfloat16()
    dY = torch.randn(M, N, device=dev).bfloat16()
    gW = torch.empty(N, K, device=dev)
    gWt = torch.empty(K, N, device=dev)
    dA = torch.empty(M, K, device=dev).bfloat16()
    Y = torch.empty(M, N, device=dev).bfloat16()
    fl = 2 * M * N * K
    cases = {
        "fwd_linear": lambda: torch.nn.functional.linear(A, W, b),
        "fwd_addmm_out": lambda: torch.addmm(b, A, W.t(), out=Y),
        "fwd_transposed": lambda: torch.mm(W, A.t()),
        "wgrad_f32out": lambda: torch.mm(dY.t(), A, out_dtype=torch.float32, out=gW),
        "wgrad_bf16out": lambda: torch.mm(dY.t(), A),
        "wgrad_T_f32out": lambda: torch.mm(A.t(), dY, out_dtype=torch.float32, out=gWt),
        "dgrad": lambda: torch.mm(dY, W, out=dA),
        "dgrad_T": lambda: torch.mm(W.t(), dY.t()),
        "bias_sum": lambda: torch.sum(dY, dim=0, dtype=torch.float32),
    }
    for lib in ("cublaslt", "cublas"):
        try:
            torch.backends.cuda.preferred_blas_library(lib)
        except Exception as e:
            print(json.dumps({"lib": lib, "error": str(e)[:200]}))
            continue
        for name, fn in cases.items():
            try:
                us = timeit(fn)
                print(json.dumps({"lib": lib, "case": name, "us": round(us, 1),
                                  "tflops": round(fl / us / 1e6, 1) if name != "bias_sum" else None}), flush=True)
            except Exception as e:
                print(json.dumps({"lib": lib, "case": name, "error": str(e)[:200]}), flush=True)


if __name__ == "__main__":
    main()
