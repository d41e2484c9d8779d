#!/usr/bin/env python3
"""Time the hand-written MFMA FC GEMM (csrc/hip/fc_gemm.hip) against hipBLASLt (TunableOp choices when
the shipped file exists), plain and with the fused HDCE-loss epilogue, at the flagship shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import FcNmse, fc_linear  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.nmse import StreamNMSE  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import use_tuned_gemms  # noqa: E402


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
    print("tuned gemms:", use_tuned_gemms())
    dev = torch.device("cuda")
    E, U, B, N, K, Ns = 3, 3, 256, 2048, 4096, 18000
    M, S = E * U * B, E * U
    A = torch.randn(M, K, device=dev).bfloat16()
    W = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    L = torch.randn(S, Ns, N, device=dev)
    P = L + 0.1 * torch.randn_like(L)
    idx = torch.randperm(Ns, device=dev)[:B]
    u = torch.arange(U, device=dev).view(U, 1, 1)
    e = torch.arange(E, device=dev).view(1, 1, E)
    rowoff = ((e * U + u).expand(U, B, E) * Ns + idx.view(1, B, 1)).reshape(-1).to(torch.int32)
    rowden = torch.stack([L.reshape(-1, N)[rowoff.long()].pow(2).sum(1), P.reshape(-1, N)[rowoff.long()].pow(2).sum(1)],
                         1).contiguous()
    nm = StreamNMSE(HDCEModel.row_stream(E, U, B, dev), S, N)
    nm.rowoff = rowoff
    bg = torch.empty(N, device=dev)
    op = FcNmse(M, N, K, (E, U, B), dev)
    loss = torch.zeros(2, device=dev)
    skip = torch.zeros(1, device=dev)
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2 * M * N * K
    res = {
        "hipblaslt_linear": timeit(lambda: torch.nn.functional.linear(A, W, b)),
        "hand_linear": timeit(lambda: fc_linear(A, W, b, out=Y)),
        "hipblaslt_linear+nmse_fused": timeit(lambda: nm.fused(torch.nn.functional.linear(A, W, b), L, P, bg, (E, U, B),
                                                               rowden=rowden)),
        "hand_fc_nmse": timeit(lambda: op(A, W, b, L, P, rowoff, rowden, bg, loss, skip)),
    }
    import ctypes
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    f = nat.fn(nat.hip_lib(), "qd_fc_gemm_diag", [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 + [ctypes.c_void_p])
    for dbg, name in ((1, "hand_no_loads"), (2, "hand_no_mfma")):
        res[name] = timeit(lambda: nat.check(f(nat.ptr(A), nat.ptr(W), nat.ptr(Y), M, N, K, dbg,
                                               nat.stream_ptr(dev)), "diag"))
    for k, v in res.items():
        print(f"{k:28s} {v:7.1f} us   {fl / v / 1e6:7.1f} TFLOP/s")


if __name__ == "__main__":
    main()
