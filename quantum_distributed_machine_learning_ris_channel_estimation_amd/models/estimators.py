"""Estimator / classifier modules with the reference's class names and state_dict keys.

Reference: Estimators_QuantumNAT_onchipQNN.py
  DCE_P128  E:40-75     flat deep channel estimator (Conv stack + FC in one module)
  SC_P128   E:79-101    classical scenario classifier
  QSC_P128  E:107-228   hybrid CNN -> VQC -> linear scenario classifier
  Conv_P128 E:237-268   per-scenario feature extractor
  FC_P128   E:272-279   shared feature mapper 4096 -> 2048
  NMSE_cuda / NMSELoss  E:282-295

Layer indices inside ``nn.Sequential`` containers, parameter names and registration
order are kept identical so checkpoints load in both directions (SURVEY.md §2.1
"Checkpoint keys").  The compute behind them is MI355X-native: the quantum layer runs
on the HIP state-vector kernels (ops/quantum.py), the classical layers through the
fused kernels in ops/ when driven by the training engines (train/engine.py).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.quantum import qsim, init_weights_

PILOT_GRID = {128: (16, 8), 256: (16, 16)}  # P128 is the reference grid (R:108); P256 is ours


def pilot_grid(pilot_num: int):
    if pilot_num not in PILOT_GRID:
        raise ValueError(f"unsupported Pilot_num {pilot_num}; known: {sorted(PILOT_GRID)}")
    return PILOT_GRID[pilot_num]


def _cnn_stack(features: int = 32, kernel_size: int = 3, padding: int = 1) -> nn.Sequential:
    layers = [nn.Conv2d(2, features, kernel_size, stride=1, padding=padding, bias=False),
              nn.BatchNorm2d(features), nn.ReLU(inplace=True)]
    for _ in range(2):
        layers += [nn.Conv2d(features, features, kernel_size, stride=1, padding=padding, bias=False),
                   nn.BatchNorm2d(features), nn.ReLU(inplace=True)]
    return nn.Sequential(*layers)


class DCE_P128(nn.Module):
    """Flat estimator: 3x[conv3x3 -> BN -> ReLU] then Linear(32*H*W, 2048) (E:40-75)."""

    def __init__(self, pilot_num: int = 128, out_dim: int = 64 * 16 * 2):
        super().__init__()
        self.features, self.kernel_size, self.padding = 32, 3, 1
        self.H, self.W = pilot_grid(pilot_num)
        self.cnn = _cnn_stack(self.features, self.kernel_size, self.padding)
        self.FC = nn.Linear(self.features * self.H * self.W, out_dim)

    def forward(self, x):
        x = self.cnn(x)
        return self.FC(x.reshape(x.shape[0], self.features * self.H * self.W))


class SC_P128(nn.Module):
    """Classical scenario classifier (E:79-101): conv-relu-pool x2 -> Linear -> log_softmax."""

    def __init__(self, pilot_num: int = 128, n_classes: int = 3):
        super().__init__()
        H, W = pilot_grid(pilot_num)
        self.pilot_num = pilot_num
        self.flat = 32 * (H // 4) * (W // 4)
        self.conv1 = nn.Conv2d(2, 32, kernel_size=3, padding=1, bias=False)
        self.conv2 = nn.Conv2d(32, 32, kernel_size=3, padding=1, bias=False)
        self.FC = nn.Linear(self.flat, n_classes)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.conv1(x)), 2, 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2, 2)
        return F.log_softmax(self.FC(x.reshape(x.shape[0], self.flat)), dim=1)


class QuantumLayer(nn.Module):
    """Drop-in for PennyLane's ``qml.qnn.TorchLayer`` (E:144-149): owns ``weights``
    of shape (n_layers, n_qubits, 2), maps (B, n) angles to (B, n) <Z_i> values."""

    def __init__(self, n_qubits: int, n_layers: int, backend: Optional[str] = None):
        super().__init__()
        self.n_qubits, self.n_layers = n_qubits, n_layers
        self.backend = backend
        self.weights = nn.Parameter(init_weights_(torch.empty(n_layers, n_qubits, 2)))

    def forward(self, x: torch.Tensor, weights: Optional[torch.Tensor] = None) -> torch.Tensor:
        w = self.weights if weights is None else weights
        return qsim(x.float(), w, self.backend)

    def extra_repr(self) -> str:
        return f"n_qubits={self.n_qubits}, n_layers={self.n_layers}, backend={self.backend}"


class QSC_P128(nn.Module):
    """Quantum scenario classifier (E:107-228).

    preprocess CNN -> tanh angles -> VQC (<Z_i>) -> Linear(n, n_classes) -> log_softmax.

    QuantumNAT (E:175-199): the reference perturbs the qlayer parameters in place,
    runs the forward, and restores them *before* backward, so autograd mixes noisy
    intermediates with clean leaves.  Here the semantics are explicit: forward AND
    backward use w + noise_level*N(0,1); the gradient is applied to the clean master
    weights (straight-through), and the master weights are never mutated.
    On-chip gradient pruning (E:205-228) zeroes every gradient with |g| <= threshold
    for ALL parameters (classical included), as the reference does.
    ``use_quantum=False`` selects ``classical_fallback`` (referenced at E:168-170 but never
    defined there): Linear(n, n) + Tanh in place of the VQC, an equal-width classical ablation
    with the same (-1, 1) output range as <Z_i>.
    """

    def __init__(self, n_qubits: int = 6, n_layers: int = 3, n_classes: int = 3, use_quantumnat: bool = True,
                 use_gradient_pruning: bool = True, pilot_num: int = 128, backend: Optional[str] = None,
                 noise_level: float = 0.01, gradient_threshold: float = 0.1, use_quantum: bool = True):
        super().__init__()
        self.use_quantum = use_quantum
        self.num_qubits = n_qubits
        self.n_layers = n_layers
        self.n_classes = n_classes
        self.use_quantumnat = use_quantumnat
        self.use_gradient_pruning = use_gradient_pruning
        self.noise_level = noise_level if use_quantumnat else 0.0
        self.gradient_threshold = gradient_threshold
        self.last_pruning_ratio = 0.0
        H, W = pilot_grid(pilot_num)
        flat = 32 * (H // 4) * (W // 4)
        # registration order matters: qlayer.weights is the first state_dict key (E:149 < E:152)
        self.qlayer = QuantumLayer(n_qubits, n_layers, backend)
        self.preprocess = nn.Sequential(
            nn.Conv2d(2, 16, kernel_size=3, stride=1, padding=1),
            nn.ReLU(),
            nn.MaxPool2d(2),
            nn.Conv2d(16, 32, kernel_size=3, stride=1, padding=1),
            nn.ReLU(),
            nn.MaxPool2d(2),
            nn.Flatten(),
            nn.Linear(flat, n_qubits),
            nn.Tanh(),
        )
        self.classifier = nn.Linear(n_qubits, n_classes)
        if not use_quantum:
            self.classical_fallback = nn.Sequential(nn.Linear(n_qubits, n_qubits), nn.Tanh())

    def quantum_weights(self, generator: Optional[torch.Generator] = None) -> torch.Tensor:
        w = self.qlayer.weights
        if self.training and self.use_quantumnat and self.noise_level > 0:
            noise = torch.randn(w.shape, device=w.device, dtype=w.dtype, generator=generator)
            return w + self.noise_level * noise
        return w

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        angles = self.preprocess(x)
        if self.use_quantum:
            xq = self.qlayer(angles, self.quantum_weights())
        else:
            xq = self.classical_fallback(angles)
        return F.log_softmax(self.classifier(xq), dim=1)

    @torch.no_grad()
    def apply_gradient_pruning(self, sync_stats: bool = True) -> None:
        """g *= (|g| > threshold) for every parameter (E:205-228)."""
        if not self.use_gradient_pruning:
            return
        total, pruned = 0, None
        for p in self.parameters():
            if p.grad is None:
                continue
            mask = p.grad.abs() > self.gradient_threshold
            cnt = (~mask).sum()
            pruned = cnt if pruned is None else pruned + cnt
            total += p.grad.numel()
            p.grad.mul_(mask)
        if sync_stats and total > 0 and pruned is not None:
            ratio = pruned.item() / total
            self.last_pruning_ratio = ratio
            if ratio > 0.1:
                print(f"Gradient pruning: {ratio:.1%} gradients pruned")


class Conv_P128(nn.Module):
    """Per-scenario feature extractor (E:237-268): (B,2,H,W) -> (B, 32*H*W), C-major flatten."""

    def __init__(self, pilot_num: int = 128):
        super().__init__()
        self.features, self.kernel_size, self.padding = 32, 3, 1
        self.H, self.W = pilot_grid(pilot_num)
        self.cnn = _cnn_stack(self.features, self.kernel_size, self.padding)

    def forward(self, x):
        x = self.cnn(x)
        return x.reshape(x.shape[0], self.features * self.H * self.W)


class FC_P128(nn.Module):
    """Shared feature mapper Linear(32*H*W -> 2048) (E:272-279)."""

    def __init__(self, pilot_num: int = 128, out_dim: int = 64 * 16 * 2):
        super().__init__()
        H, W = pilot_grid(pilot_num)
        self.FC = nn.Linear(32 * H * W, out_dim)

    def forward(self, x):
        return self.FC(x)


def NMSE_cuda(x_hat: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """Batch-global NMSE: sum((x_hat-x)^2) / sum(x^2) over the WHOLE tensor (E:282-286)."""
    x_hat = x_hat.float()
    x = x.float()
    return torch.sum((x_hat - x) ** 2) / torch.sum(x ** 2)


class NMSELoss(nn.Module):
    def forward(self, x_hat, x):
        return NMSE_cuda(x_hat, x)
