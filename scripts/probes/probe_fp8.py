#!/usr/bin/env python3
"""Probe fp8 GEMM support on the MI355X (gfx950): torch._scaled_mm with OCP e4m3 / e5m2 operands
at the FC_P128 shapes, accuracy vs fp32 and time vs bf16.  Prints JSON lines."""
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
    print(json.dumps({"device": torch.cuda.get_device_name(0),
                      "arch": getattr(torch.cuda.get_device_properties(0), "gcnArchName", "?")}))
    M, K, N = 2304, 4096, 2048   # FC rows = 9 streams x 256 samples
    torch.manual_seed(0)
    A = torch.randn(M, K, device=dev) * 0.5
    W = torch.randn(N, K, device=dev) * 0.02
    ref = A @ W.t()
    A16, W16 = A.bfloat16(), W.bfloat16()
    t_bf = timeit(lambda: torch.mm(A16, W16.t()))
    err_bf = float((torch.mm(A16, W16.t()).float() - ref).norm() / ref.norm())
    print(json.dumps({"op": "bf16_mm", "us": round(t_bf, 1), "tflops": round(2 * M * N * K / t_bf / 1e6, 1),
                      "rel_err": err_bf}))
    for name in ("float8_e4m3fn", "float8_e4m3fnuz", "float8_e5m2"):
        dt = getattr(torch, name, None)
        if dt is None:
            continue
        try:
            fmax = torch.finfo(dt).max
            sa = (A.abs().max() / fmax).float().reshape(())
            sw = (W.abs().max() / fmax).float().reshape(())
            A8 = (A / sa).to(dt)
            W8 = (W / sw).to(dt)
            f = lambda: torch._scaled_mm(A8, W8.t(), scale_a=sa, scale_b=sw, out_dtype=torch.bfloat16)
            out = f()
            t = timeit(f)
            err = float((out.float() - ref).norm() / ref.norm())
            print(json.dumps({"op": f"scaled_mm_{name}", "us": round(t, 1), "tflops": round(2 * M * N * K / t / 1e6, 1),
                              "rel_err": err}))
        except Exception as e:
            print(json.dumps({"op": f"scaled_mm_{name}", "error": f"{type(e).__name__}: {str(e)[:300]}"}))


if __name__ == "__main__":
    main()
