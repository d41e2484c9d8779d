#!/usr/bin/env python3
"""Time the HDCE loss + gradient pass: the one-pass kernel (qd_nmse_fused, several rows-per-block
choices) against the three-kernel path (row sums + reduce/finalize, grad_bias + slab sum)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.nmse import StreamNMSE  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel  # noqa: E402


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
    E, U, B, cols, N = 3, 3, 256, 2048, 18000
    S = E * U
    L = torch.randn(S, N, cols, device=dev)
    P = L + 0.1 * torch.randn_like(L)
    idx = torch.randperm(N, device=dev)[:B]
    u = torch.arange(U, device=dev).view(U, 1, 1)
    e = torch.arange(E, device=dev).view(1, 1, E)
    rowoff = ((e * U + u).expand(U, B, E) * N + idx.view(1, B, 1)).reshape(-1).to(torch.int32)
    rs = HDCEModel.row_stream(E, U, B, dev)
    Y = torch.randn(U * B * E, cols, device=dev).bfloat16()
    nm = StreamNMSE(rs, S, cols)
    nm.rowoff = rowoff
    bg = torch.empty(cols, device=dev)

    def old():
        nm.sums_finalize(Y, L, P)
        nm.grad_bias(Y, L, bg, out_dtype=torch.bfloat16)

    res = {"three_kernels": timeit(old)}
    for m in (1, 2, 4, 8):
        res[f"fused_rpc{E * m}"] = timeit(lambda: nm.fused(Y, L, P, bg, (E, U, B), rpc_mult=m))
    # the same rows gathered into contiguous buffers first (rowoff = identity): what the random
    # 8 KB-row reads out of the 2 x 1.3 GB label stores cost
    Lg = L.view(-1, cols)[rowoff.long()].contiguous()
    Pg = P.view(-1, cols)[rowoff.long()].contiguous()
    nm.rowoff = torch.arange(U * B * E, device=dev, dtype=torch.int32)
    res["fused_rpc6_contiguous"] = timeit(lambda: nm.fused(Y, Lg.view(S, -1, cols), Pg.view(S, -1, cols), bg, (E, U, B), rpc_mult=2))
    nm.rowoff = rowoff
    # a pre-gather copy itself (torch index_select of both stores)
    res["torch_pregather_copy"] = timeit(lambda: (torch.index_select(L.view(-1, cols), 0, rowoff.long(), out=Lg),
                                                  torch.index_select(P.view(-1, cols), 0, rowoff.long(), out=Pg)))
    for k, v in res.items():
        print(f"{k:22s} {v:7.1f} us")


if __name__ == "__main__":
    main()
