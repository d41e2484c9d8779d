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


def gemm_wgrad_ok(M: int, N: int, K: int, cfg: int = 0) -> bool:
    """dW (N, K) = dY (M, N)^T A (M, K): does tile configuration ``cfg`` cover this shape?"""
    return bool(_gemm_fn("qd_gemm_wgrad_ok", [_i, _i, _i, _i])(M, N, K, cfg))


def gemm_dgrad_ok(M: int, N: int, K: int, cfg: int = 0) -> bool:
    """dA (M, K) = dY (M, N) W (N, K): does tile configuration ``cfg`` cover this shape?"""
    return bool(_gemm_fn("qd_gemm_dgrad_ok", [_i, _i, _i, _i])(M, N, K, cfg))


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


def gemm_dgrad_bnred(dY: torch.Tensor, W: torch.Tensor, out: torch.Tensor, cfg: int, z: torch.Tensor,
                     st: torch.Tensor, part: torch.Tensor, B: int, U: int, HW: int) -> torch.Tensor:
    """gemm_dgrad with the last conv layer's BN backward reduction in the epilogue (csrc/hip/gemm.hip BnRedEpi):
    part (U, M / 144, 2, 96) receives per (group, tile) sum g / sum g xhat of g = dA [a z + b > 0] -- the partial
    rows csrc/hip/conv.hip bn_bwd_reduce_kernel would write.  z: the layer's pre-BN output in dA's layout;
    st: its BN records (U, 96, 8).  3 experts, cfg 0, 2, 5 or 6."""
    M, N = dY.shape
    K = W.shape[1]
    assert dY.dtype == W.dtype == z.dtype == torch.bfloat16 and dY.is_contiguous() and W.is_contiguous()
    assert z.is_contiguous() and z.numel() == M * K and part.is_contiguous() and part.numel() == U * (M // 144) * 2 * 96
    f = _gemm_fn("qd_gemm_dgrad_bnred", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _i, _i, _i, _p])
    nat.check(f(nat.ptr(dY), nat.ptr(W), nat.ptr(out), M, N, K, cfg, nat.ptr(z), nat.ptr(st), nat.ptr(part), B, U, HW,
                nat.stream_ptr(W.device)), "gemm_dgrad_bnred")
    return out


def gemm_fwd_f8(A8: torch.Tensor, W8: torch.Tensor, deq: torch.Tensor, b: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, cfg: int = 1) -> torch.Tensor:
    """Y (M, N) bf16 = deq[0] deq[1] A8 W8^T (+ b): OCP e4m3 operands (torch.float8_e4m3fn, row-major,
    K % 128 == 0), fp32 accumulation (csrc/hip/gemm.hip qd_gemm_fwd_bias_f8).  cfg 1: the MX-scaled
    MFMA (v_mfma_scale_f32_16x16x128_f8f6f4, unit block scales, K % 256 == 0); 2: the same with producer waves;
    0: mfma_f32_16x16x32_fp8_fp8."""
    M, K = A8.shape
    N = W8.shape[0]
    assert A8.dtype == W8.dtype == torch.float8_e4m3fn and A8.is_contiguous() and W8.is_contiguous()
    assert deq.dtype == torch.float32 and deq.numel() >= 2
    if cfg >= 1 and K % 256:
        cfg = 0
    Y = out if out is not None else torch.empty(M, N, device=A8.device, dtype=torch.bfloat16)
    f = _gemm_fn("qd_gemm_fwd_bias_f8", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p])
    nat.check(f(nat.ptr(A8), nat.ptr(W8), nat.ptr(deq), nat.ptr(b) if b is not None else None, nat.ptr(Y), M, N, K,
                cfg, nat.stream_ptr(A8.device)), "gemm_fwd_bias_f8")
    return Y


def gemm_nt_f8(P8: torch.Tensor, Q8: torch.Tensor, sP: torch.Tensor, sQ: torch.Tensor, out: Optional[torch.Tensor] = None,
               out_dtype=torch.bfloat16, cfg: int = 1) -> torch.Tensor:
    """C (I, J) = sP sQ P8 Q8^T on the MX-scaled e4m3 MFMA (csrc/hip/gemm.hip qd_gemm_nt_f8): P8 (I, K), Q8 (J, K)
    row-major e4m3, sP / sQ one-element device scales, C fp32 or bf16.  cfg 1: 144 x 128 tiles, 2: 128 x 256."""
    I, K = P8.shape
    J = Q8.shape[0]
    assert P8.dtype == Q8.dtype == torch.float8_e4m3fn and P8.is_contiguous() and Q8.is_contiguous() and Q8.shape[1] == K
    assert sP.dtype == sQ.dtype == torch.float32 and sP.is_cuda and sQ.is_cuda
    C = out if out is not None else torch.empty(I, J, device=P8.device, dtype=out_dtype)
    assert C.dtype in (torch.float32, torch.bfloat16) and C.shape == (I, J) and C.stride(1) == 1
    f = _gemm_fn("qd_gemm_nt_f8", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p])
    nat.check(f(nat.ptr(P8), nat.ptr(Q8), nat.ptr(sP), nat.ptr(sQ), nat.ptr(C), I, J, K, C.stride(0),
                int(C.dtype == torch.float32), cfg, nat.stream_ptr(P8.device)), "gemm_nt_f8")
    return C


def transpose_u8(src: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(C, R) = (R, C)^T for a 1-byte tensor (e4m3 operand copies), R % 64 == 0, C % 256 == 0."""
    R, C = src.shape
    assert src.element_size() == 1 and src.is_contiguous()
    dst = out if out is not None else torch.empty(C, R, device=src.device, dtype=src.dtype)
    assert dst.shape == (C, R) and dst.is_contiguous() and dst.dtype == src.dtype
    f = _gemm_fn("qd_transpose_u8", [_p, _p, _i, _i, _p])
    nat.check(f(nat.ptr(src), nat.ptr(dst), R, C, nat.stream_ptr(src.device)), "transpose_u8")
    return dst


def gemm_wgrad_f8(dY8: torch.Tensor, A8: torch.Tensor, s_dy: torch.Tensor, s_a: torch.Tensor,
                  out: torch.Tensor, cfg: int = 0) -> torch.Tensor:
    """dW (N, K) fp32 = s_dy s_a dY8^T A8 from the row-major e4m3 dY8 (M, N) and A8 (M, K) (MX-scaled MFMA, both
    operands read i-contiguous through ds_read_b64_tr_b8: csrc/hip/gemm.hip qd_gemm_wgrad_f8).  M % 256 == 0.
    (``cfg`` is accepted for symmetry with gemm_dgrad_f8: one tile configuration.)"""
    M, N = dY8.shape
    K = A8.shape[1]
    assert dY8.dtype == A8.dtype == torch.float8_e4m3fn and dY8.is_contiguous() and A8.is_contiguous()
    assert A8.shape[0] == M and out.dtype == torch.float32 and out.shape == (N, K) and out.stride(1) == 1
    f = _gemm_fn("qd_gemm_wgrad_f8", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p])
    nat.check(f(nat.ptr(dY8), nat.ptr(A8), nat.ptr(s_dy), nat.ptr(s_a), nat.ptr(out), M, N, K, out.stride(0), cfg,
                nat.stream_ptr(dY8.device)), "gemm_wgrad_f8")
    return out


def gemm_dgrad_f8(dY8: torch.Tensor, W8: torch.Tensor, s_dy: torch.Tensor, s_w: torch.Tensor,
                  out: Optional[torch.Tensor] = None, cfg: int = 0) -> torch.Tensor:
    """dA (M, K) bf16 = s_dy s_w dY8 W8 from the row-major e4m3 dY8 (M, N) and W8 (N, K) (csrc/hip/gemm.hip
    qd_gemm_dgrad_f8).  N % 256 == 0, M % 144 == 0.  cfg 1: the same tiles with producer waves."""
    M, N = dY8.shape
    K = W8.shape[1]
    assert dY8.dtype == W8.dtype == torch.float8_e4m3fn and dY8.is_contiguous() and W8.is_contiguous()
    assert W8.shape[0] == N
    dA = out if out is not None else torch.empty(M, K, device=dY8.device, dtype=torch.bfloat16)
    assert dA.dtype == torch.bfloat16 and dA.shape == (M, K) and dA.is_contiguous()
    f = _gemm_fn("qd_gemm_dgrad_f8", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p])
    nat.check(f(nat.ptr(dY8), nat.ptr(W8), nat.ptr(s_dy), nat.ptr(s_w), nat.ptr(dA), M, N, K, cfg,
                nat.stream_ptr(dY8.device)), "gemm_dgrad_f8")
    return dA


def gemm_dgrad_f8_bnred(dY8: torch.Tensor, W8: torch.Tensor, s_dy: torch.Tensor, s_w: torch.Tensor, out: torch.Tensor,
                        cfg: int, z: torch.Tensor, st: torch.Tensor, part: torch.Tensor, B: int, U: int,
                        HW: int) -> torch.Tensor:
    """gemm_dgrad_f8 with gemm_dgrad_bnred's epilogue (csrc/hip/gemm.hip qd_gemm_dgrad_f8_bnred): the e4m3 data
    gradient also writes layer 3's BN backward partial rows.  HW == 128, M == U B 3, 3 B >= 144; cfg 1 or 0."""
    M, N = dY8.shape
    K = W8.shape[1]
    assert dY8.dtype == W8.dtype == torch.float8_e4m3fn and dY8.is_contiguous() and W8.is_contiguous()
    assert W8.shape[0] == N and out.dtype == torch.bfloat16 and out.shape == (M, K) and out.is_contiguous()
    assert z.dtype == torch.bfloat16 and z.is_contiguous() and z.numel() == M * K
    assert part.is_contiguous() and part.numel() == U * (M // 144) * 2 * 96
    f = _gemm_fn("qd_gemm_dgrad_f8_bnred", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _i, _i, _i, _p])
    nat.check(f(nat.ptr(dY8), nat.ptr(W8), nat.ptr(s_dy), nat.ptr(s_w), nat.ptr(out), M, N, K, cfg, nat.ptr(z),
                nat.ptr(st), nat.ptr(part), B, U, HW, nat.stream_ptr(dY8.device)), "gemm_dgrad_f8_bnred")
    return out

