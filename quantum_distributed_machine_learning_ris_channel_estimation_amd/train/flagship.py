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

from .. import _native as nat
from ..data.datasets import DMLStore, make_dml_stores
from ..models.estimators import QSC_P128
from ..ops.gather import StepGather
from ..ops.optim import FlatParamSpace, make_optimizer
from ..ops.slabsum import SlabBatch
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
    split_graphs: bool = False   # force the 3-graph DP execution plan even at world 1 (testing)
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
        self.hdce.attach_fc_shadow(self.hopt)   # after the broadcast: the shadow starts in sync
        self.qopt = make_optimizer(self.qspace, "adamw", cfg.lr, weight_decay=cfg.qsc_weight_decay,
                                   prune_thr=0.1 if cfg.use_gradient_pruning else 0.0)
        sp = self.hdce.space
        n_conv = sp.offsets[sp.names.index("CE.FC.weight")]
        self.hstep = HDCEStep(self.hdce, self.U, self.B)
        # NaN guard: the NMSE kernel sets the flag, the QSC head adds to it; it travels in the small
        # bucket so every rank sees the same (summed) flag and skips -- or steps -- in lockstep
        self.skip = self.hstep.skip
        self.cstep = ClassifierStep(self.qsc, self.S, space=self.qspace, batch_total=self.S * self.B, skip=self.skip)
        self.cstep.writes_grads = self.cstep.hip is not None
        # bucket "fc": 33.6 MB, ready first; bucket "small": conv + QSC grads + skip flag, coalesced
        self.buckets = GradBuckets(ctx, {"fc": [sp.grad[n_conv:]],
                                         "small": [sp.grad[:n_conv], self.qspace.grad, self.skip]})
        self.idx = torch.zeros(self.B, dtype=torch.long, device=dev)
        self.gat = StepGather(self.E, self.U, self.B, self.hdce.H, self.hdce.W, dev, with_classifier=True)
        self.perm = torch.randperm(self.store.n, device=dev)
        self.cursor = 0
        # the loss kernels' own static buffers double as the step's loss outputs (no per-step copies)
        self.hloss = self.hstep.nmse.loss
        self.qloss = self.cstep.hip.loss if self.cstep.hip is not None else torch.zeros(1, device=dev)
        self.labels = self.store.scen.repeat_interleave(self.B)
        self.slabs = SlabBatch()
        graphs = cfg.hip_graphs and dev.type == "cuda"
        if ctx.world == 1 and not cfg.split_graphs:
            # one graph: gather, both forwards, NMSE, both backwards, both optimizers
            self.graphs = [GraphedStep(self._step_body, enabled=graphs)]
        else:
            # three graphs around the two gradient all-reduces; the FC bucket (33.6 MB) is reduced on
            # RCCL's stream while graph 2 (conv + QSC backward) runs on the compute stream
            pool = torch.cuda.graph_pool_handle() if graphs else None
            self.graphs = [GraphedStep(f, enabled=graphs, pool=pool) for f in (self._phase1, self._phase2, self._phase3)]

    # -- phases ---------------------------------------------------------------------------
    def _phase1(self) -> None:
        # the fused GPU kernels WRITE every gradient (one producer per element): no zero_grad fills
        if not self.hstep.writes_grads:
            self.hdce.space.zero_grad()
        if not self.cstep.writes_grads:
            self.qspace.zero_grad()
        self.gat(self.store, self.idx)           # one launch: conv input, classifier input, label rows
        loss = self.hstep.forward_fc_gathered(self.gat, self.store)
        if loss is not self.hloss:
            self.hloss.copy_(loss)

    def _phase2(self) -> None:
        # every gradient-slab reduction of the phase (3 conv weight slabs, the quantum layer's and the
        # QSC preprocess slab) goes out as ONE launch when both steps write (overwrite) their grads
        share = self.hstep.hip and self.cstep.hip is not None and self.cstep.writes_grads and self.hstep.writes_grads
        slabs = self.slabs if share else None
        self.hstep.backward_conv(slabs=slabs)
        q = self.cstep(self.gat.xq, self.labels, slabs=slabs)
        if slabs is not None:
            slabs.launch(accumulate=False, stream=nat.stream_ptr(self.ctx.device))
        if q is not self.qloss:
            self.qloss.copy_(q)

    def _phase3(self) -> None:
        g = 1.0 / self.ctx.world
        self.hopt.step(grad_scale=g, skip=self.skip)
        self.qopt.step(grad_scale=g, skip=self.skip)

    def _step_body(self) -> None:
        self._phase1()
        self.buckets.launch("fc")
        self._phase2()
        self.buckets.launch("small")
        self.buckets.wait()
        self._phase3()

    @property
    def graphed(self) -> GraphedStep:
        return self.graphs[0]

    def next_batch(self) -> None:
        if self.cursor + self.B > self.store.n:
            self.perm = torch.randperm(self.store.n, device=self.ctx.device)
            self.cursor = 0
        self.idx.copy_(self.perm[self.cursor:self.cursor + self.B])
        self.cursor += self.B

    def step(self) -> None:
        self.next_batch()
        if len(self.graphs) == 1:
            self.graphs[0]()
            return
        g1, g2, g3 = self.graphs
        g1()
        self.buckets.launch("fc")
        g2()
        self.buckets.launch("small")
        self.buckets.wait()
        g3()

    @property
    def samples_per_step(self) -> int:
        return self.S * self.B
