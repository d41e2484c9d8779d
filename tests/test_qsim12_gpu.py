"""The 12-qubit simulator on the matrix cores (csrc/hip/qsim12_mfma.hip): forward <Z>, the adjoint's dx and the
summed weight gradient against the fp64 C++ oracle (csrc/cpu/qsim_cpu.cpp through ops.quantum.qsim "cpu") and
against qsim_big.hip's VALU kernels, with and without QuantumNAT weight groups."""
import ctypes
import math

import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.quantum import qsim

pytestmark = pytest.mark.gpu
_p, _i = ctypes.c_void_p, ctypes.c_int
N = 12


def _mfma12(x, w, gE, wgroup):
    """(E, dx, dw summed over the slab rows) from qd_qsim_mfma12_fwd / _bwd; w (G, L, 12, 2) or (L, 12, 2)."""
    lib = nat.hip_lib()
    B = x.shape[0]
    L = w.shape[-3]
    G = w.shape[0] if w.dim() == 4 else 1
    dev = x.device
    wsb = nat.fn(lib, "qd_qsim_mfma12_workspace", [_i, _i], ctypes.c_longlong)(G, L)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    ps = torch.empty(B * (8 << N), dtype=torch.uint8, device=dev)
    rows = nat.fn(lib, "qd_qsim_big_grid", [_i])(B)
    E = torch.empty(B, N, device=dev)
    dx = torch.empty(B, N, device=dev)
    slab = torch.full((rows, 2 * N * L), float("nan"), device=dev)
    st = nat.stream_ptr(dev)
    f = nat.fn(lib, "qd_qsim_mfma12_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
    b = nat.fn(lib, "qd_qsim_mfma12_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
    nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(E), B, N, L, wgroup, nat.ptr(ws), nat.ptr(ps), st), "mfma12 fwd")
    nat.check(b(nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, N, L, wgroup, nat.ptr(ws),
                nat.ptr(ps), st), "mfma12 bwd")
    torch.cuda.synchronize()
    return E, dx, slab.sum(0).view(L, N, 2)


@pytest.mark.parametrize("L,B", [(1, 5), (2, 7), (3, 9), (5, 4)])
def test_qsim12_mfma_matches_cpp(cuda, L, B):
    g = torch.Generator().manual_seed(11 * L + B)
    x = torch.rand(B, N, generator=g) * 2 - 1
    w = torch.rand(L, N, 2, generator=g) * 2 * math.pi
    gE = torch.randn(B, N, generator=g)
    xc, wc = x.clone().requires_grad_(), w.clone().requires_grad_()
    Ec = qsim(xc, wc, "cpu")
    (Ec * gE).sum().backward()
    E, dx, dw = _mfma12(x.to(cuda), w.to(cuda), gE.to(cuda), 0)
    assert torch.allclose(E.cpu(), Ec, atol=5e-5), float((E.cpu() - Ec).abs().max())
    assert torch.allclose(dx.cpu(), xc.grad, atol=2e-4), float((dx.cpu() - xc.grad).abs().max())
    assert torch.allclose(dw.cpu(), wc.grad, atol=1e-3), float((dw.cpu() - wc.grad).abs().max())


def test_qsim12_mfma_groups_matches_cpp(cuda):
    """QuantumNAT weight groups (w (G, L, 12, 2), sample s uses group s / wgroup): the slab sums every group."""
    G, b, L = 3, 4, 3
    g = torch.Generator().manual_seed(5)
    x = torch.rand(G * b, N, generator=g) * 2 - 1
    w = torch.rand(G, L, N, 2, generator=g) * 6.28
    gE = torch.randn(G * b, N, generator=g)
    Ec, dxc, dwc = [], [], torch.zeros(L, N, 2, dtype=torch.float64)
    for i in range(G):
        xi, wi = x[i * b:(i + 1) * b].clone().requires_grad_(), w[i].clone().requires_grad_()
        Ei = qsim(xi, wi, "cpu")
        (Ei * gE[i * b:(i + 1) * b]).sum().backward()
        Ec.append(Ei.detach())
        dxc.append(xi.grad)
        dwc += wi.grad.double()
    E, dx, dw = _mfma12(x.to(cuda), w.to(cuda), gE.to(cuda), b)
    assert torch.allclose(E.cpu(), torch.cat(Ec), atol=5e-5)
    assert torch.allclose(dx.cpu(), torch.cat(dxc), atol=2e-4)
    assert torch.allclose(dw.cpu().double(), dwc, atol=1e-3), float((dw.cpu().double() - dwc).abs().max())


@pytest.mark.parametrize("B,G", [(1000, 1), (2304, 9)])
def test_qsim12_mfma_matches_valu_kernels(cuda, B, G):
    """Flagship-sized batches (grid-stride over 512 workgroups, 9 QuantumNAT groups) against qsim_big.hip's
    kernels on the same inputs: E, dx and the summed weight gradient."""
    lib = nat.hip_lib()
    L = 3
    torch.manual_seed(B)
    x = torch.rand(B, N, device=cuda) * 3.0
    w = torch.rand(G, L, N, 2, device=cuda) * 6.28
    gE = torch.randn(B, N, device=cuda) / B
    wgroup = B // G if G > 1 else 0
    E, dx, dw = _mfma12(x, w, gE, wgroup)
    rows = nat.fn(lib, "qd_qsim_big_grid", [_i])(B)
    E0, dx0 = torch.empty(B, N, device=cuda), torch.empty(B, N, device=cuda)
    slab0 = torch.empty(rows, 2 * N * L, device=cuda)
    ps = torch.empty(B * (8 << N), dtype=torch.uint8, device=cuda)
    st = nat.stream_ptr(cuda)
    nat.check(nat.fn(lib, "qd_qsim_big_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])(
        nat.ptr(x), nat.ptr(w), nat.ptr(E0), B, N, L, wgroup, None, nat.ptr(ps), st), "big fwd")
    nat.check(nat.fn(lib, "qd_qsim_big_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])(
        nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx0), nat.ptr(slab0), B, N, L, wgroup, None, nat.ptr(ps), st),
        "big bwd")
    torch.cuda.synchronize()
    dw0 = slab0.sum(0).view(L, N, 2)
    assert torch.allclose(E, E0, atol=5e-5), float((E - E0).abs().max())
    assert torch.allclose(dx, dx0, atol=2e-4 / 100), float((dx - dx0).abs().max())
    assert torch.allclose(dw, dw0, atol=1e-4), float((dw - dw0).abs().max())


def test_qsim12_mfma_deterministic(cuda):
    """Two runs on the same inputs give bit-identical outputs (fixed-order reductions, no atomics)."""
    torch.manual_seed(3)
    B, L = 600, 3
    x = torch.rand(B, N, device=cuda)
    w = torch.rand(L, N, 2, device=cuda) * 6.28
    gE = torch.randn(B, N, device=cuda)
    a = _mfma12(x, w, gE, 0)
    b = _mfma12(x, w, gE, 0)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def _bwd8(x, w, gE, wgroup, mfma):
    """8 qubits: the register forward (qsim.hip, keeps psi_final) then the MFMA adjoint (qd_qsim_mfma8_bwd) or the
    register adjoint (qd_qsim_bwd_saved) -> (E, dx, dw summed over the slab rows)."""
    lib = nat.hip_lib()
    B, n = x.shape
    L = w.shape[-3]
    G = w.shape[0] if w.dim() == 4 else 1
    dev = x.device
    ps = torch.empty(B * (8 << n), dtype=torch.uint8, device=dev)
    rows = nat.fn(lib, "qd_qsim_bwd_grid", [_i, _i])(n, B)
    E = torch.empty(B, n, device=dev)
    dx = torch.empty(B, n, device=dev)
    slab = torch.full((rows, 2 * n * L), float("nan"), device=dev)
    st = nat.stream_ptr(dev)
    nat.check(nat.fn(lib, "qd_qsim_fwd_save", [_p, _p, _p, _i, _i, _i, _i, _p, _p])(
        nat.ptr(x), nat.ptr(w), nat.ptr(E), B, n, L, wgroup, nat.ptr(ps), st), "fwd_save")
    if mfma:
        wsb = nat.fn(lib, "qd_qsim_mfma8_workspace", [_i, _i], ctypes.c_longlong)(G, L)
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        nat.check(nat.fn(lib, "qd_qsim_mfma8_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])(
            nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, n, L, wgroup, nat.ptr(ws), nat.ptr(ps),
            st), "mfma8 bwd")
    else:
        nat.check(nat.fn(lib, "qd_qsim_bwd_saved", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p])(
            nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, n, L, wgroup, nat.ptr(ps), st),
            "bwd_saved")
    torch.cuda.synchronize()
    return E, dx, slab.sum(0).view(L, n, 2)


@pytest.mark.parametrize("L,B", [(1, 5), (3, 9), (4, 33)])
def test_qsim8_mfma_adjoint_matches_cpp(cuda, L, B):
    g = torch.Generator().manual_seed(3 * L + B)
    x = torch.rand(B, 8, generator=g) * 2 - 1
    w = torch.rand(L, 8, 2, generator=g) * 2 * math.pi
    gE = torch.randn(B, 8, generator=g)
    xc, wc = x.clone().requires_grad_(), w.clone().requires_grad_()
    (qsim(xc, wc, "cpu") * gE).sum().backward()
    _, dx, dw = _bwd8(x.to(cuda), w.to(cuda), gE.to(cuda), 0, True)
    assert torch.allclose(dx.cpu(), xc.grad, atol=5e-5), float((dx.cpu() - xc.grad).abs().max())
    assert torch.allclose(dw.cpu(), wc.grad, atol=5e-4), float((dw.cpu() - wc.grad).abs().max())


@pytest.mark.parametrize("B,G", [(2304, 9), (5000, 1)])
def test_qsim8_mfma_adjoint_matches_register_kernel(cuda, B, G):
    """Flagship batch (9 QuantumNAT groups; and > 4096 samples: waves loop over samples) against qsim.hip's
    register-resident adjoint on the same saved states."""
    torch.manual_seed(B)
    L = 3
    x = torch.rand(B, 8, device=cuda) * 3.0
    w = torch.rand(G, L, 8, 2, device=cuda) * 6.28
    gE = torch.randn(B, 8, device=cuda) / B
    wgroup = B // G if G > 1 else 0
    _, dx, dw = _bwd8(x, w, gE, wgroup, True)
    _, dx0, dw0 = _bwd8(x, w, gE, wgroup, False)
    assert torch.allclose(dx, dx0, atol=1e-6), float((dx - dx0).abs().max())
    assert torch.allclose(dw, dw0, atol=1e-5), float((dw - dw0).abs().max())
