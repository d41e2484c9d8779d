"""Hand-written MFMA FC_P128 GEMMs (csrc/hip/gemm.hip): the training forward with the HDCE loss fused
into its epilogue (dY, per-row error partials, bias-gradient partials; Y never written), the weight
and data gradients, and the inference forward (bias, optional expert-routed rows).

Reference: FC_P128 (Estimators_QuantumNAT_onchipQNN.py:272-279) + NMSE_cuda (E:282-286) per stream
(Runner_P128_QuantumNAT_onchipQNN.py:109-113, 194-199).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from .. import _native as nat

_p, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float


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


def gemm_wgrad_adam(dY: torch.Tensor, A: torch.Tensor, opt, lo: int, slot: int, skip: Optional[torch.Tensor] = None,
                    grad_scale: float = 1.0, cfg: int = 0, shape=None) -> None:
    """dW = dY^T A with the Adam step of the flat range ``[lo, lo + N*K)`` of ``opt`` (ops.optim.FusedOptimizer,
    its ``fuse_range`` slot ``slot``) applied in the GEMM's epilogue: the weight, moments and the bf16 shadow
    are updated, dW itself is never stored (csrc/hip/gemm.hip qd_gemm_wgrad_adam)."""
    M, N = dY.shape
    K = A.shape[1]
    assert dY.dtype == A.dtype == torch.bfloat16 and dY.is_contiguous() and A.is_contiguous() and A.shape[0] == M
    assert opt.kind == "adam" and opt.fused == (lo, lo + N * K)
    sp = opt.space
    sh = None
    if opt.shadow is not None:
        assert opt.shadow_lo <= lo and lo + N * K <= opt.shadow_hi
        sh = ctypes.c_void_p(opt.shadow.data_ptr() + 2 * (lo - opt.shadow_lo))
    f = _gemm_fn("qd_gemm_wgrad_adam", [_p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _f, _f, _f, _f, _p, _i, _p])
    at = lambda t: ctypes.c_void_p(t.data_ptr() + 4 * lo)
    nat.check(f(nat.ptr(dY), nat.ptr(A), M, N, K, K, at(sp.flat), at(opt.m), at(opt.v), sh, nat.ptr(opt.lr_t),
                nat.ptr(opt.step_t[slot:]), nat.ptr(skip) if skip is not None else None, opt.betas[0], opt.betas[1],
                opt.eps, grad_scale, nat.ptr(opt.done[slot:]), cfg, nat.stream_ptr(A.device)), "gemm_wgrad_adam")


def gemm_dgrad(dY: torch.Tensor, W: torch.Tensor, out: Optional[torch.Tensor] = None, cfg: int = 0) -> torch.Tensor:
    """dA = dY W, bf16 (dY (M, N), W (N, K) row-major; the reduction runs over N)."""
    M, N = dY.shape
    K = W.shape[1]
    assert dY.dtype == W.dtype == torch.bfloat16 and dY.is_contiguous() and W.is_contiguous() and W.shape[0] == N
    dA = out if out is not None else torch.empty(M, K, device=W.device, dtype=torch.bfloat16)
    f = _gemm_fn("qd_gemm_dgrad", [_p, _p, _p, _i, _i, _i, _i, _p])
    nat.check(f(nat.ptr(dY), nat.ptr(W), nat.ptr(dA), M, N, K, cfg, nat.stream_ptr(W.device)), "gemm_dgrad")
    return dA


def gemm_fwd_f8(A8: torch.Tensor, W8: torch.Tensor, deq: torch.Tensor, b: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Y (M, N) bf16 = deq[0] deq[1] A8 W8^T (+ b): OCP e4m3 operands (torch.float8_e4m3fn, row-major,
    K % 128 == 0), fp32 accumulation (csrc/hip/gemm.hip qd_gemm_fwd_bias_f8, mfma_f32_16x16x32_fp8_fp8)."""
    M, K = A8.shape
    N = W8.shape[0]
    assert A8.dtype == W8.dtype == torch.float8_e4m3fn and A8.is_contiguous() and W8.is_contiguous()
    assert deq.dtype == torch.float32 and deq.numel() >= 2
    Y = out if out is not None else torch.empty(M, N, device=A8.device, dtype=torch.bfloat16)
    f = _gemm_fn("qd_gemm_fwd_bias_f8", [_p, _p, _p, _p, _p, _i, _i, _i, _p])
    nat.check(f(nat.ptr(A8), nat.ptr(W8), nat.ptr(deq), nat.ptr(b) if b is not None else None, nat.ptr(Y), M, N, K,
                nat.stream_ptr(A8.device)), "gemm_fwd_bias_f8")
    return Y
