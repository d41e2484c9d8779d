"""Quantum layer: three independent implementations vs a dense NumPy oracle + exact invariants.

The oracle builds every gate as a full 2^n x 2^n matrix with PennyLane's wire convention
(wire 0 = most significant qubit), so it shares no indexing code with the C++ simulator
(wire i = bit i), the torch reference or the HIP kernels.  PennyLane itself is not
installable here: parity with it is pinned through this oracle of its documented gate
definitions (RY, RZ, CNOT, AngleEmbedding(rotation='Y'), expval(PauliZ)).
"""
import math

import numpy as np
import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.quantum import qsim

I2 = np.eye(2)
Z = np.diag([1.0, -1.0])


def ry(t):
    c, s = math.cos(t / 2), math.sin(t / 2)
    return np.array([[c, -s], [s, c]], dtype=complex)


def rz(p):
    return np.diag([np.exp(-0.5j * p), np.exp(0.5j * p)])


def on_wire(U, w, n):
    mats = [U if i == w else I2 for i in range(n)]
    out = mats[0]
    for m in mats[1:]:
        out = np.kron(out, m)
    return out


def cnot(c, t, n):
    D = 1 << n
    M = np.zeros((D, D))
    for k in range(D):
        bits = [(k >> (n - 1 - i)) & 1 for i in range(n)]  # wire i = MSB-first
        if bits[c]:
            bits[t] ^= 1
        j = sum(b << (n - 1 - i) for i, b in enumerate(bits))
        M[j, k] = 1
    return M


def oracle(x, w):
    n, L = x.shape[0], w.shape[0]
    psi = np.zeros(1 << n, dtype=complex)
    psi[0] = 1
    for i in range(n):
        psi = on_wire(ry(x[i]), i, n) @ psi
    for l in range(L):
        for i in range(n):
            psi = on_wire(ry(w[l, i, 0]), i, n) @ psi
            psi = on_wire(rz(w[l, i, 1]), i, n) @ psi
        for i in range(n - 1):
            psi = cnot(i, i + 1, n) @ psi
        psi = cnot(n - 1, 0, n) @ psi
    return np.array([np.real(np.conj(psi) @ on_wire(Z, i, n) @ psi) for i in range(n)])


@pytest.mark.parametrize("backend", ["cpu", "torch"])
@pytest.mark.parametrize("n,L", [(2, 1), (3, 2), (4, 3), (5, 1), (6, 3)])
def test_forward_matches_dense_oracle(backend, n, L):
    rng = np.random.default_rng(n * 10 + L)
    x = rng.uniform(-1, 1, (4, n))
    w = rng.uniform(0, 2 * np.pi, (L, n, 2))
    E = qsim(torch.tensor(x, dtype=torch.float32), torch.tensor(w, dtype=torch.float32), backend).numpy()
    ref = np.stack([oracle(x[b], w) for b in range(4)])
    np.testing.assert_allclose(E, ref, atol=2e-6)


@pytest.mark.parametrize("n,L", [(2, 1), (4, 3), (6, 2)])
def test_backward_matches_parameter_shift(n, L):
    """Parameter shift (f(t+pi/2) - f(t-pi/2))/2 is EXACT for RY/RZ generators."""
    rng = np.random.default_rng(7 + n)
    x = rng.uniform(-1, 1, (3, n))
    w = rng.uniform(0, 2 * np.pi, (L, n, 2))
    g = rng.normal(size=(3, n))
    xt = torch.tensor(x, dtype=torch.float32, requires_grad=True)
    wt = torch.tensor(w, dtype=torch.float32, requires_grad=True)
    (qsim(xt, wt, "cpu") * torch.tensor(g, dtype=torch.float32)).sum().backward()

    def f(xx, ww):
        return sum(float(g[b] @ oracle(xx[b], ww)) for b in range(3))

    for idx in np.ndindex(*w.shape):
        wp, wm = w.copy(), w.copy()
        wp[idx] += np.pi / 2
        wm[idx] -= np.pi / 2
        assert abs((f(x, wp) - f(x, wm)) / 2 - float(wt.grad[idx])) < 2e-4
    for b in range(3):
        for i in range(n):
            xp, xm = x.copy(), x.copy()
            xp[b, i] += np.pi / 2
            xm[b, i] -= np.pi / 2
            assert abs((f(xp, w) - f(xm, w)) / 2 - float(xt.grad[b, i])) < 2e-4


def test_last_layer_rz_has_zero_gradient():
    """Only permutations follow the last RZs before a diagonal measurement -> dL/dw[L-1,:,1] == 0."""
    torch.manual_seed(0)
    x = torch.rand(5, 4) * 2 - 1
    w = (torch.rand(3, 4, 2) * 6.28).requires_grad_()
    qsim(x, w, "cpu").pow(2).sum().backward()
    assert w.grad[-1, :, 1].abs().max() < 1e-6
    assert w.grad[:-1].abs().max() > 1e-3


def test_first_layer_ry_adds_to_embedding_angle():
    torch.manual_seed(1)
    x = torch.rand(6, 5) * 2 - 1
    w = torch.rand(2, 5, 2) * 6.28
    d = torch.rand(5) * 0.3
    w2 = w.clone()
    w2[0, :, 0] += d
    assert torch.allclose(qsim(x, w2, "cpu"), qsim(x + d, w, "cpu"), atol=1e-6)


def test_grouped_weights_cpu_equals_per_group():
    torch.manual_seed(2)
    G, b, n, L = 3, 4, 4, 2
    x = torch.rand(G * b, n)
    w = torch.rand(G, L, n, 2) * 6
    E = qsim(x, w, "cpu")
    for g in range(G):
        assert torch.allclose(E[g * b:(g + 1) * b], qsim(x[g * b:(g + 1) * b], w[g], "cpu"))


def test_cpu_config_4_qubit_2_class_batch32_trains():
    """BASELINE config 1: 4-qubit VQC scenario classifier, 2-class, CPU state-vector sim, batch 32."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import QSC_P128
    torch.manual_seed(0)
    m = QSC_P128(n_qubits=4, n_layers=3, n_classes=2, use_quantumnat=True, use_gradient_pruning=False)
    x = torch.randn(32, 2, 16, 8)
    y = (x[:, 0].mean((1, 2)) > 0).long()
    x[y == 1] += 0.5
    opt = torch.optim.AdamW(m.parameters(), lr=1e-2, weight_decay=0.01)
    losses = []
    for _ in range(40):
        opt.zero_grad()
        loss = torch.nn.functional.nll_loss(m(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] * 0.8
