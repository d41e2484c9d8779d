#!/usr/bin/env python3
"""Round 5: the FC GEMMs with producer waves (gemm.hip Geo PW = 4) against the shipped tiles, at the flagship shape
M=2304, N=2048, K=4096.  Each variant is first checked against an fp32 torch product (max |err| / max |ref|), then
timed: rounds interleave the variants in one process, median and min over rounds are printed.

    python scripts/probes/probe_gemm_r5.py [rounds]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import (  # noqa: E402
    gemm_dgrad, gemm_dgrad_bnred, gemm_dgrad_f8, gemm_dgrad_f8_bnred, gemm_fwd, gemm_fwd_f8, gemm_wgrad, gemm_wgrad_f8)


def timeit(fn, iters=40):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M, N, K = 2304, 2048, 4096
    A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    W = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
    dY = (torch.rand(M, N, device=dev) * 2 - 1).bfloat16()
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    dW = torch.empty(N, K, device=dev)
    dA = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    fl = 2 * M * N * K
    ref = {"fwd": (A.float() @ W.float().t()), "wgrad": (dY.float().t() @ A.float()), "dgrad": (dY.float() @ W.float())}
    out = {"fwd": Y, "wgrad": dW, "dgrad": dA}
    var = {}
    for c in (6, 2, 0, 7, 8, 9, 10):
        var[f"fwd_c{c}"] = ("fwd", lambda c=c: gemm_fwd(A, W, None, out=Y, cfg=c))
    for c in (1, 0, 5, 6, 7):
        var[f"wgrad_c{c}"] = ("wgrad", lambda c=c: gemm_wgrad(dY, A, out=dW, cfg=c))
    for c in (2, 0, 5, 6):
        var[f"dgrad_c{c}"] = ("dgrad", lambda c=c: gemm_dgrad(dY, W, out=dA, cfg=c))
    # e4m3 (fp8 estimator): MX-scaled MFMA, shipped tiles vs the same with producer waves
    A8, W8, dY8 = A.to(torch.float8_e4m3fn), W.to(torch.float8_e4m3fn), dY.to(torch.float8_e4m3fn)
    one, deq = torch.ones(1, device=dev), torch.ones(2, device=dev)
    ref["fwd8"] = A8.float() @ W8.float().t()
    ref["wgrad8"] = dY8.float().t() @ A8.float()
    ref["dgrad8"] = dY8.float() @ W8.float()
    out["fwd8"], out["wgrad8"], out["dgrad8"] = Y, dW, dA
    for c in (1, 2):
        var[f"fwd8_c{c}"] = ("fwd8", lambda c=c: gemm_fwd_f8(A8, W8, deq, None, out=Y, cfg=c))
    for c in (0, 1):
        var[f"wgrad8_c{c}"] = ("wgrad8", lambda c=c: gemm_wgrad_f8(dY8, A8, one, one, out=dW, cfg=c))
        var[f"dgrad8_c{c}"] = ("dgrad8", lambda c=c: gemm_dgrad_f8(dY8, W8, one, one, out=dA, cfg=c))
    # the data gradients with layer 3's BN backward reduction in the epilogue (B 256, U 3, HW 128: M = 2304)
    z = torch.randn(M, K, device=dev).bfloat16()
    st = torch.rand(3, 96, 8, device=dev)
    part = torch.empty(3 * (M // 144) * 2 * 96, device=dev)
    var["dgrad_bnred_c6"] = ("dgrad", lambda: gemm_dgrad_bnred(dY, W, dA, 6, z, st, part, 256, 3, 128))
    # (diagnosis) the bf16 epilogue with its z loads replaced by a constant (d1), without the cross-lane / cross-wave
    # reduction (d2), both (d3)
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops import fc as _fc
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as _nat
    fdbg = _fc._gemm_fn("qd_gemm_dgrad_bnred_dbg", [_fc._p, _fc._p, _fc._p] + [_fc._i] * 4 + [_fc._p] * 3 + [_fc._i] * 3
                        + [_fc._p])
    for d in (1, 2, 3):
        var[f"dgrad_bnred_d{d}"] = ("dgrad", lambda d=d: _nat.check(fdbg(
            _nat.ptr(dY), _nat.ptr(W), _nat.ptr(dA), M, N, K, d, _nat.ptr(z), _nat.ptr(st), _nat.ptr(part), 256, 3,
            128, _nat.stream_ptr(dY.device)), "dbg"))
    for c in (0, 1):
        var[f"dgrad8_bnred_c{c}"] = ("dgrad8", lambda c=c: gemm_dgrad_f8_bnred(dY8, W8, one, one, dA, c, z, st, part,
                                                                               256, 3, 128))
    if only:
        var = {k: v for k, v in var.items() if any(k.startswith(o) for o in only)}
    bad = []
    for name, (kind, fn) in var.items():
        out[kind].zero_()
        fn()
        torch.cuda.synchronize()
        r = ref[kind]
        err = float((out[kind].float() - r).abs().max() / r.abs().max())
        ok = err < 2e-2
        print(f"check {name:14s} rel max err {err:.2e} {'ok' if ok else 'BAD'}", flush=True)
        if not ok:
            bad.append(name)
    var = {k: v for k, v in var.items() if k not in bad}
    ts = {k: [] for k in var}
    for _ in range(rounds):
        for k, (_, fn) in var.items():
            ts[k].append(timeit(fn))
    for k, v in ts.items():
        md = statistics.median(v)
        print(f"{k:14s} median {md:8.2f} us  min {min(v):8.2f} us  {fl / md * 1e-6:7.1f} TF/s", flush=True)
    if bad:
        print("BAD:", ",".join(bad))
        sys.exit(1)


if __name__ == "__main__":
    main()
