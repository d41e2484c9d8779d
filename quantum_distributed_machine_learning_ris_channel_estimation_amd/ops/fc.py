"""Hand-written MFMA FC_P128 GEMM (csrc/hip/fc_gemm.hip) with the HDCE loss fused into its epilogue.

Reference: FC_P128 (Estimators_QuantumNAT_onchipQNN.py:272-279) + NMSE_cuda (E:282-286) per stream
(Runner_P128_QuantumNAT_onchipQNN.py:109-113, 194-199).

``fc_linear(A, W, b)``             Y = A W^T + b, bf16 (tile 144 x 128, one workgroup per CU)
``FcNmse(...)(A, W, b, ...)``      the training forward: the GEMM epilogue turns the accumulator
                                   straight into dY = 2 (Y - L) / (S den_s) (bf16), per-row error
                                   partials and per-tile bias-gradient partials; one small finish
                                   launch forms loss / loss_perf / the NaN flag / the bias gradient.
                                   Y is never written to memory.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from .. import _native as nat

_p, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float


def tile_m(M: int, N: int, K: int) -> int:
    """M tile the kernel uses for this shape (144 or 128), 0 if unsupported."""
    return int(nat.fn(nat.hip_lib(), "qd_fc_gemm_tile_m", [_i, _i, _i])(M, N, K))


def fc_linear(A: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    M, K = A.shape
    N = W.shape[0]
    assert A.dtype == W.dtype == torch.bfloat16 and A.is_contiguous() and W.is_contiguous() and W.shape[1] == K
    assert b is None or (b.dtype == torch.bfloat16 and b.numel() == N and b.is_contiguous())
    if not tile_m(M, N, K):
        raise ValueError(f"fc_linear: shape {(M, N, K)} not supported")
    Y = out if out is not None else torch.empty(M, N, device=A.device, dtype=torch.bfloat16)
    f = nat.fn(nat.hip_lib(), "qd_fc_gemm_bias", [_p, _p, _p, _p, _i, _i, _i, _p])
    nat.check(f(nat.ptr(A), nat.ptr(W), nat.ptr(b) if b is not None else None, nat.ptr(Y), M, N, K,
                nat.stream_ptr(A.device)), "fc_gemm_bias")
    return Y


class FcNmse:
    """FC forward + per-stream NMSE loss + dY + bias gradient for rows in (u, b, e) order.

    ``layout`` = (E, U, B); labels (S, N_store, cols) read in place through ``rowoff`` (int32, one
    store row per output row); ``rowden`` (M, 2) fp32 per-row label / perf powers (ops/gather.py)."""

    def __init__(self, M: int, N: int, K: int, layout, device):
        self.M, self.N, self.K = M, N, K
        self.E, self.U, self.B = layout
        assert M == self.E * self.U * self.B
        self.tm = tile_m(M, N, K)
        if not self.tm:
            raise ValueError(f"FcNmse: shape {(M, N, K)} not supported")
        S = self.E * self.U
        self.dY = torch.empty(M, N, device=device, dtype=torch.bfloat16)
        self.rowpart = torch.empty(M, N // 128, 2, device=device)
        self.colpart = torch.empty(M // self.tm, N, device=device)
        self.ss = torch.zeros(S, 4, device=device)
        self._f = nat.fn(nat.hip_lib(), "qd_fc_gemm_nmse", [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                                                            _i, _i, _i, _i, _i, _i, _f, _p])

    @staticmethod
    def supported(M: int, N: int, K: int) -> bool:
        return bool(tile_m(M, N, K)) and N % 64 == 0

    def __call__(self, A, W, b, label, perf, rowoff, rowden, bias_grad, loss, skip, loss_scale: float = 1.0):
        assert A.shape == (self.M, self.K) and W.shape == (self.N, self.K)
        assert A.dtype == W.dtype == torch.bfloat16 and A.is_contiguous() and W.is_contiguous()
        assert label.dtype == torch.float32 and label.stride(-1) == 1 and label.shape[-1] == self.N
        assert rowoff.dtype == torch.int32 and rowoff.numel() == self.M and rowden.shape == (self.M, 2)
        nat.check(self._f(nat.ptr(A), nat.ptr(W), nat.ptr(b) if b is not None else None, nat.ptr(label),
                          nat.ptr(perf) if perf is not None else None, nat.ptr(rowoff), nat.ptr(rowden),
                          nat.ptr(self.dY), nat.ptr(self.rowpart), nat.ptr(self.colpart), nat.ptr(bias_grad),
                          nat.ptr(self.ss), nat.ptr(loss), nat.ptr(skip) if skip is not None else None,
                          self.M, self.N, self.K, self.E, self.U, self.B, loss_scale, nat.stream_ptr(A.device)),
                  "fc_gemm_nmse")
        return self.dY


# ---------------------------------------------------------------------------------------------------
# csrc/hip/gemm.hip: the hand-written forward / weight-gradient / data-gradient GEMMs of FC_P128
# (cfg selects a tile configuration; 0 = the default chosen by measurement, see gemm.hip's header)

def _gemm_fn(name, argtypes):
    return nat.fn(nat.hip_lib(), name, argtypes)


def gemm_fwd_ok(M: int, N: int, K: int, cfg: int = 0) -> bool:
    return bool(_gemm_fn("qd_gemm_fwd_ok", [_i, _i, _i, _i])(M, N, K, cfg))


def gemm_tile_m(cfg: int = 0) -> int:
    return int(_gemm_fn("qd_gemm_tile_m", [_i])(cfg))


def gemm_fwd(A: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
             cfg: int = 0, expert: Optional[torch.Tensor] = None, n_experts: int = 0) -> torch.Tensor:
    """Y = A W^T (+ b), bf16 (A (M_A, K), W (N, K) row-major).  ``expert`` ((M,) int64, values <
    ``n_experts``): row i of the product uses A[i * n_experts + expert[i]] -- expert-routed rows, the
    selection fused into the GEMM's operand loads (A holds every expert's features per sample)."""
    M, K = A.shape
    N = W.shape[0]
    if expert is not None:
        assert expert.dtype == torch.int64 and expert.is_contiguous() and expert.device == A.device
        M = expert.numel()
        assert A.shape[0] >= M * n_experts
    assert A.dtype == W.dtype == torch.bfloat16 and A.is_contiguous() and W.is_contiguous() and W.shape[1] == K
    assert b is None or (b.dtype == torch.bfloat16 and b.numel() == N and b.is_contiguous())
    if not gemm_fwd_ok(M, N, K, cfg):
        raise ValueError(f"gemm_fwd: shape {(M, N, K)} not supported by cfg {cfg}")
    Y = out if out is not None else torch.empty(M, N, device=A.device, dtype=torch.bfloat16)
    f = _gemm_fn("qd_gemm_fwd_bias", [_p, _p, _p, _p, _i, _i, _i, _i, _p, _i, _p])
    nat.check(f(nat.ptr(A), nat.ptr(W), nat.ptr(b) if b is not None else None, nat.ptr(Y), M, N, K, cfg,
                nat.ptr(expert) if expert is not None else None, n_experts, nat.stream_ptr(A.device)), "gemm_fwd_bias")
    return Y


def gemm_wgrad(dY: torch.Tensor, A: torch.Tensor, out: Optional[torch.Tensor] = None, cfg: int = 0) -> torch.Tensor:
    """dW = dY^T A in fp32 (dY (M, N), A (M, K) bf16 row-major; the reduction runs over M)."""
    M, N = dY.shape
    K = A.shape[1]
    assert dY.dtype == A.dtype == torch.bfloat16 and dY.is_contiguous() and A.is_contiguous() and A.shape[0] == M
    W = out if out is not None else torch.empty(N, K, device=A.device, dtype=torch.float32)
    assert W.dtype == torch.float32 and W.shape == (N, K) and W.stride(1) == 1
    f = _gemm_fn("qd_gemm_wgrad", [_p, _p, _p, _i, _i, _i, _i, _i, _p])
    nat.check(f(nat.ptr(dY), nat.ptr(A), nat.ptr(W), M, N, K, W.stride(0), cfg, nat.stream_ptr(A.device)),
              "gemm_wgrad")
    return W


def gemm_dgrad(dY: torch.Tensor, W: torch.Tensor, out: Optional[torch.Tensor] = None, cfg: int = 0) -> torch.Tensor:
    """dA = dY W, bf16 (dY (M, N), W (N, K) row-major; the reduction runs over N)."""
    M, N = dY.shape
    K = W.shape[1]
    assert dY.dtype == W.dtype == torch.bfloat16 and dY.is_contiguous() and W.is_contiguous() and W.shape[0] == N
    dA = out if out is not None else torch.empty(M, K, device=W.device, dtype=torch.bfloat16)
    f = _gemm_fn("qd_gemm_dgrad", [_p, _p, _p, _i, _i, _i, _i, _p])
    nat.check(f(nat.ptr(dY), nat.ptr(W), nat.ptr(dA), M, N, K, cfg, nat.stream_ptr(W.device)), "gemm_dgrad")
    return dA
