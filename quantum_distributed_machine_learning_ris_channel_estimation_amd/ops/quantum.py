"""Variational-quantum-circuit layer: expectation values <Z_i> of the QSC circuit.

Reference behaviour: ``QSC_P128.qlayer`` = PennyLane ``TorchLayer`` over a
``default.qubit`` QNode (Estimators_QuantumNAT_onchipQNN.py:121-149): AngleEmbedding
RY(x_i), then per layer RY(w[l,i,0]) RZ(w[l,i,1]) on every wire and a CNOT ring,
measured as [<Z_0>, ..., <Z_{n-1}>].  PennyLane differentiates it by backprop
through its tape ("best" diff method, E:148).

Here three interchangeable backends implement the SAME function:

* ``hip``   -- hand-written CDNA4 kernels: csrc/hip/qsim.hip (n <= 10: register-resident
               state, one wave per sample) and csrc/hip/qsim_big.hip (n = 11..16: one
               512-thread workgroup per sample, state in LDS or an HBM workspace),
               forward + adjoint backward.  Default on GPU.
* ``cpu``   -- C++/OpenMP simulator (csrc/cpu/qsim_cpu.cpp). Default on CPU.
* ``torch`` -- eager complex-tensor simulator differentiated by autograd: the
               "reference-equivalent" gate-by-gate path used as a baseline and an
               oracle.  Never selected implicitly on a GPU.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import torch

from .. import _native as nat

_i = ctypes.c_int
_f = ctypes.c_float
_p = ctypes.c_void_p

HIP_REG_MAX_QUBITS = 10   # register-resident kernel
HIP_MAX_QUBITS = 16       # workgroup-per-sample kernel above that


def stream_sim_ok(n: int, L: int) -> bool:
    """(n, L) runs on the streamed simulator (csrc/hip/qsim_stream.hip: n = 13..16, L >= 2, one
    workgroup per (sample, 4096-amplitude brick) per pass); else qsim_big.hip's workgroup-per-sample
    kernels run it."""
    return bool(nat.fn(nat.hip_lib(), "qd_qsim_stream_ok", [_i, _i])(n, L))


def _stream_ws(n: int, B: int, L: int, backward: bool, device) -> torch.Tensor:
    nbytes = nat.fn(nat.hip_lib(), "qd_qsim_stream_workspace", [_i, _i, _i, _i], ctypes.c_longlong)(n, B, L,
                                                                                                 int(backward))
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def _big_ws(n: int, grid: int, backward: bool, device) -> Optional[torch.Tensor]:
    nbytes = nat.fn(nat.hip_lib(), "qd_qsim_big_workspace", [_i, _i, _i], ctypes.c_longlong)(n, grid, int(backward))
    return torch.empty(nbytes, dtype=torch.uint8, device=device) if nbytes else None


def hip_qsim_fwd(x: torch.Tensor, w: torch.Tensor, E: torch.Tensor, wgroup: int = 0) -> None:
    """Raw launcher (no autograd): E = <Z>(x, w); x (B, n) fp32, w (L, n, 2) or (G, L, n, 2) fp32."""
    lib = nat.hip_lib()
    B, n = x.shape
    L = w.shape[-3]
    st = nat.stream_ptr(x.device)
    if n <= HIP_REG_MAX_QUBITS:
        f = nat.fn(lib, "qd_qsim_fwd", [_p, _p, _p, _i, _i, _i, _i, _p])
        nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(E), B, n, L, wgroup, st), "qd_qsim_fwd")
        return
    if stream_sim_ok(n, L):
        ws = _stream_ws(n, B, L, False, x.device)
        f = nat.fn(lib, "qd_qsim_stream_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
        nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(E), B, n, L, wgroup, nat.ptr(ws), None, st), "qd_qsim_stream_fwd")
        return
    grid = nat.fn(lib, "qd_qsim_big_grid", [_i])(B)
    ws = _big_ws(n, grid, False, x.device)
    f = nat.fn(lib, "qd_qsim_big_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
    nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(E), B, n, L, wgroup, nat.ptr(ws) if ws is not None else None, None,
                st), "qd_qsim_big_fwd")


def hip_qsim_bwd_slab(x: torch.Tensor, w: torch.Tensor, gE: torch.Tensor, dx: torch.Tensor) -> torch.Tensor:
    """Raw adjoint backward: writes dx (B, n), returns the (rows, 2nL) weight-grad slab."""
    lib = nat.hip_lib()
    B, n = x.shape
    L = w.shape[-3]
    P = 2 * n * L
    st = nat.stream_ptr(x.device)
    if n <= HIP_REG_MAX_QUBITS:
        rows = nat.fn(lib, "qd_qsim_bwd_grid", [_i, _i])(n, B)
        slab = torch.empty(rows, P, device=x.device, dtype=torch.float32)
        f = nat.fn(lib, "qd_qsim_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p])
        nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, n, L, wgroup_of(x, w), st),
                  "qd_qsim_bwd")
        return slab
    if stream_sim_ok(n, L):
        slab = torch.empty(nat.fn(lib, "qd_qsim_stream_rows", [_i])(B), P, device=x.device, dtype=torch.float32)
        ws = _stream_ws(n, B, L, True, x.device)
        f = nat.fn(lib, "qd_qsim_stream_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
        nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, n, L, wgroup_of(x, w),
                    nat.ptr(ws), None, st), "qd_qsim_stream_bwd")
        return slab
    rows = nat.fn(lib, "qd_qsim_big_grid", [_i])(B)
    slab = torch.empty(rows, P, device=x.device, dtype=torch.float32)
    ws = _big_ws(n, rows, True, x.device)
    f = nat.fn(lib, "qd_qsim_big_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
    nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, n, L, wgroup_of(x, w),
                nat.ptr(ws) if ws is not None else None, None, st), "qd_qsim_big_bwd")
    return slab


def wgroup_of(x: torch.Tensor, w: torch.Tensor) -> int:
    return x.shape[0] // w.shape[0] if w.dim() == 4 else 0


# ----------------------------------------------------------------------------- HIP
class _QSimHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor, wgroup: int = 0):
        B, n = x.shape
        x = x.detach().float().contiguous()
        w = w.detach().float().contiguous()
        E = torch.empty(B, n, device=x.device, dtype=torch.float32)
        if B > 0:
            hip_qsim_fwd(x, w, E, wgroup)
        ctx.save_for_backward(x, w)
        return E

    @staticmethod
    def backward(ctx, gE: torch.Tensor):
        x, w = ctx.saved_tensors
        B, n = x.shape
        L = w.shape[-3]
        P = 2 * n * L
        gE = gE.float().contiguous()
        dx = torch.empty_like(x)
        dw = torch.zeros(P, device=x.device, dtype=torch.float32)
        if B > 0:
            slab = hip_qsim_bwd_slab(x, w, gE, dx)
            r = nat.fn(nat.hip_lib(), "qd_reduce_slab", [_p, _p, _i, _i, _f, _p])
            nat.check(r(nat.ptr(slab), nat.ptr(dw), slab.shape[0], P, 0.0, nat.stream_ptr(x.device)),
                      "qd_reduce_slab")
        dw = dw.view(L, n, 2)
        if w.dim() == 4:  # grouped (noisy) weights: every group maps back to the same master weights
            dw = _group_grad(dw, w)
        return dx, dw, None


def _group_grad(dw: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    # The slab already summed over all samples of all groups; the grouped weights are
    # (G, L, n, 2) = master + per-group noise, so d(master) = sum_g d(w_g).  Put the total
    # in group 0 and zeros elsewhere: autograd's sum over the expand/add restores it.
    out = torch.zeros_like(w)
    out[0] = dw
    return out


# ----------------------------------------------------------------------------- CPU (C++)
class _QSimCPU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor):
        lib = nat.cpu_lib()
        B, n = x.shape
        L = w.shape[0]
        x = x.detach().float().contiguous()
        w = w.detach().float().contiguous()
        E = torch.empty(B, n, dtype=torch.float32)
        f = nat.fn(lib, "qd_cpu_qsim_fwd", [_p, _p, _p, _i, _i, _i])
        nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(E), B, n, L), "qd_cpu_qsim_fwd")
        ctx.save_for_backward(x, w)
        return E

    @staticmethod
    def backward(ctx, gE: torch.Tensor):
        x, w = ctx.saved_tensors
        lib = nat.cpu_lib()
        B, n = x.shape
        L = w.shape[0]
        gE = gE.float().contiguous()
        dx = torch.empty_like(x)
        dw = torch.empty(L, n, 2, dtype=torch.float32)
        f = nat.fn(lib, "qd_cpu_qsim_bwd", [_p, _p, _p, _p, _p, _i, _i, _i])
        nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(dw), B, n, L), "qd_cpu_qsim_bwd")
        return dx, dw


# ----------------------------------------------------------------------------- torch reference
def ring_inverse_index(n: int) -> torch.Tensor:
    """idx[j] = f^-1(j) for the CNOT-ring basis map f (CNOT(0,1) ... CNOT(n-1,0))."""
    out = []
    for j in range(1 << n):
        k = j
        k ^= (k >> (n - 1)) & 1
        for i in range(n - 2, -1, -1):
            k ^= ((k >> i) & 1) << (i + 1)
        out.append(k)
    return torch.tensor(out, dtype=torch.long)


def z_signs(n: int, device=None, dtype=torch.float32) -> torch.Tensor:
    """(2^n, n) matrix of <k|Z_i|k> = +1/-1."""
    k = torch.arange(1 << n, device=device)
    bits = (k[:, None] >> torch.arange(n, device=device)[None, :]) & 1
    return (1 - 2 * bits).to(dtype)


def qsim_torch(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """Eager gate-by-gate simulator, differentiable through autograd (complex64)."""
    B, n = x.shape
    L = w.shape[0]
    D = 1 << n
    theta = x + w[0, :, 0]
    phi = w[0, :, 1].expand(B, n)
    ch, sh = torch.cos(theta / 2), torch.sin(theta / 2)
    cp, sp = torch.cos(phi / 2), torch.sin(phi / 2)
    c0 = torch.complex(ch * cp, -ch * sp)
    c1 = torch.complex(sh * cp, sh * sp)
    state = torch.ones(B, 1, dtype=torch.complex64, device=x.device)
    for q in range(n):  # bit q becomes the most significant so far
        state = torch.cat([state * c0[:, q:q + 1], state * c1[:, q:q + 1]], dim=1)
    perm = ring_inverse_index(n).to(x.device)
    state = state[:, perm]
    for l in range(1, L):
        for q in range(n):
            th, ph = w[l, q, 0], w[l, q, 1]
            c, s = torch.cos(th / 2), torch.sin(th / 2)
            v = state.view(B, D >> (q + 1), 2, 1 << q)
            a0, a1 = v[:, :, 0, :], v[:, :, 1, :]
            e0 = torch.complex(torch.cos(ph / 2), -torch.sin(ph / 2))
            t0 = (c * a0 - s * a1) * e0
            t1 = (s * a0 + c * a1) * e0.conj()
            state = torch.stack([t0, t1], dim=2).reshape(B, D)
        state = state[:, perm]
    probs = state.real ** 2 + state.imag ** 2
    return probs @ z_signs(n, x.device)


# ----------------------------------------------------------------------------- dispatch
def default_backend(device: torch.device) -> str:
    return "hip" if device.type == "cuda" else "cpu"


def qsim(x: torch.Tensor, w: torch.Tensor, backend: Optional[str] = None) -> torch.Tensor:
    """<Z_i> of the QSC circuit for inputs x (B, n) and weights w (L, n, 2).

    ``w`` may also be grouped, (G, L, n, 2) with B % G == 0: sample b then uses
    w[b // (B/G)] (independent QuantumNAT noise per data stream)."""
    if x.dim() != 2 or w.dim() not in (3, 4) or w.shape[-2] != x.shape[1] or w.shape[-1] != 2:
        raise ValueError(f"bad shapes x={tuple(x.shape)} w={tuple(w.shape)}")
    if w.dim() == 4 and x.shape[0] % w.shape[0]:
        raise ValueError("batch must be a multiple of the weight-group count")
    n = x.shape[1]
    if n < 2:
        raise ValueError("the CNOT ring needs n_qubits >= 2")
    be = backend if backend not in (None, "auto") else default_backend(x.device)
    if be == "hip":
        if x.device.type != "cuda":
            raise RuntimeError("hip backend needs CUDA/HIP tensors")
        if n > HIP_MAX_QUBITS:
            raise NotImplementedError(f"HIP simulators support n <= {HIP_MAX_QUBITS}")
        if 2 * n * w.shape[-3] > 256 and n > HIP_REG_MAX_QUBITS:
            raise NotImplementedError("large-n HIP simulator supports 2*n*L <= 256")
        wgroup = x.shape[0] // w.shape[0] if w.dim() == 4 else 0
        return _QSimHIP.apply(x, w, wgroup)
    if w.dim() == 4:  # host backends: run per group
        G = w.shape[0]
        return torch.cat([qsim(xc, w[g], be) for g, xc in enumerate(x.chunk(G))], dim=0)
    if be == "cpu":
        if x.device.type != "cpu":
            raise RuntimeError("cpu backend needs CPU tensors")
        return _QSimCPU.apply(x, w)
    if be == "torch":
        return qsim_torch(x, w)
    raise ValueError(f"unknown backend {be!r}")


def init_weights_(w: torch.Tensor, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """PennyLane TorchLayer default init: U[0, 2*pi)."""
    with torch.no_grad():
        w.uniform_(0.0, 2 * math.pi, generator=generator)
    return w
