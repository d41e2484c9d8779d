"""Flagship training step: the full HDCE system on one 9-stream batch.

One step = the work the reference spreads over ``train_QSC_P128`` (R:335-370) and
``train_Conv_Linear_of_HDCE`` (R:181-204) for one batch of 9 (scenario, user) streams
x 256 samples: the QSC scenario classifier (CNN preprocess -> n-qubit VQC -> linear,
NLL, AdamW, optional QuantumNAT noise and gradient pruning) and the HDCE estimator
(3 scenario experts + shared FC, per-stream NMSE, Adam), both forward + backward +
optimizer, on HBM-resident synthetic data.

Execution plan per step (world = 1): one HIP graph replay containing index gather,
both forwards, the fused NMSE, both backwards and both optimizer kernels.
World > 1: the same work eagerly, with the FC gradient bucket all-reduced on RCCL's
stream while the conv/QSC backward still runs, then the small bucket, then the
optimizers (grad averaging fused into them).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ..data.datasets import DMLStore, make_dml_stores
from ..models.estimators import QSC_P128
from ..ops.optim import FlatParamSpace, make_optimizer
from ..parallel.dp import DistContext, GradBuckets
from ..utils.profiling import GraphedStep
from .engine import ClassifierStep, HDCEModel, HDCEStep


@dataclass
class FlagshipConfig:
    pilot_num: int = 128
    n_qubits: int = 8
    n_layers: int = 3
    n_classes: int = 3
    batch: int = 256            # per stream (batch_size_DML)
    data_len: int = 20000       # per stream (train + val at 0.9)
    snr_db: int = 10
    dtype: str = "bf16"
    use_quantumnat: bool = True
    use_gradient_pruning: bool = False
    lr: float = 1e-3
    qsc_weight_decay: float = 0.01
    hip_graphs: bool = True
    seed: int = 0
    n_scenarios: int = 3
    n_users: int = 3


class FlagshipTrainer:
    def __init__(self, cfg: FlagshipConfig, ctx: DistContext):
        self.cfg, self.ctx = cfg, ctx
        dev = ctx.device
        self.store, _ = make_dml_stores(cfg.data_len, cfg.pilot_num, cfg.snr_db, 0.9, dev, synthetic=True,
                                        base_seed=cfg.seed + 1000 * ctx.rank, n_scenarios=cfg.n_scenarios,
                                        n_users=cfg.n_users)
        self.E, self.U, self.B = cfg.n_scenarios, cfg.n_users, cfg.batch
        self.S = self.E * self.U
        # --- models (weights broadcast from rank 0 once; then resident)
        torch.manual_seed(cfg.seed)
        self.hdce = HDCEModel(cfg.pilot_num, dev, cfg.dtype, cfg.n_scenarios)
        self.qsc = QSC_P128(cfg.n_qubits, cfg.n_layers, cfg.n_classes, cfg.use_quantumnat,
                            cfg.use_gradient_pruning, cfg.pilot_num).to(dev)
        self.qspace = FlatParamSpace(list(self.qsc.named_parameters()), dev)
        ctx.broadcast_(self.hdce.space.flat)
        ctx.broadcast_(self.qspace.flat)
        self.hopt = make_optimizer(self.hdce.space, "adam", cfg.lr)
        self.qopt = make_optimizer(self.qspace, "adamw", cfg.lr, weight_decay=cfg.qsc_weight_decay,
                                   prune_thr=0.1 if cfg.use_gradient_pruning else 0.0)
        sp = self.hdce.space
        n_conv = sp.offsets[sp.names.index("CE.FC.weight")]
        # bucket "fc": 33.6 MB, ready first; bucket "small": conv + QSC grads, coalesced
        self.buckets = GradBuckets(ctx, {"fc": [sp.grad[n_conv:]], "small": [sp.grad[:n_conv], self.qspace.grad]})
        self.hstep = HDCEStep(self.hdce, self.U, self.B, grad_hook=self._hdce_hook)
        self.cstep = ClassifierStep(self.qsc, self.S, space=self.qspace, batch_total=self.S * self.B)
        self.idx = torch.zeros(self.B, dtype=torch.long, device=dev)
        self.perm = torch.randperm(self.store.n, device=dev)
        self.cursor = 0
        self.hloss = torch.zeros(2, device=dev)
        self.qloss = torch.zeros(1, device=dev)
        self.labels = self.store.scen.repeat_interleave(self.B)
        self.graphed = GraphedStep(self._step_body, enabled=cfg.hip_graphs and dev.type == "cuda" and ctx.world == 1)

    def _hdce_hook(self, name: str) -> None:
        if name == "fc":
            self.buckets.launch("fc")   # overlaps the conv + QSC backward below

    def _step_body(self) -> None:
        E, U, B, S = self.E, self.U, self.B, self.S
        self.hdce.space.zero_grad()
        self.qspace.zero_grad()
        Yp, HL, HP = self.store.gather(self.idx)
        # HDCE estimator: fwd, fused NMSE, FC bwd (-> bucket "fc" launched), conv bwd
        loss = self.hstep(Yp.view(E, U, B, *Yp.shape[2:]), HL.view(E, U, B, -1), HP.view(E, U, B, -1))
        self.hloss.copy_(loss)
        # QSC scenario classifier on the same pilots
        q = self.cstep(Yp.reshape(S * B, *Yp.shape[2:]), self.labels)
        self.qloss.copy_(q)
        self.buckets.launch("small")
        self.buckets.wait()
        g = 1.0 / self.ctx.world
        self.hopt.step(grad_scale=g, skip=self.hstep.skip)
        self.qopt.step(grad_scale=g)

    def next_batch(self) -> None:
        if self.cursor + self.B > self.store.n:
            self.perm = torch.randperm(self.store.n, device=self.ctx.device)
            self.cursor = 0
        self.idx.copy_(self.perm[self.cursor:self.cursor + self.B])
        self.cursor += self.B

    def step(self) -> None:
        self.next_batch()
        self.graphed()

    @property
    def samples_per_step(self) -> int:
        return self.S * self.B
