"""Flagship training step: the full HDCE system on one 9-stream batch.

One step = the work the reference spreads over ``train_QSC_P128`` (R:335-370) and
``train_Conv_Linear_of_HDCE`` (R:181-204) for one batch of 9 (scenario, user) streams
x 256 samples: the QSC scenario classifier (CNN preprocess -> n-qubit VQC -> linear,
NLL, AdamW, optional QuantumNAT noise and gradient pruning) and the HDCE estimator
(3 scenario experts + shared FC, per-stream NMSE, Adam), both forward + backward +
optimizer, on HBM-resident synthetic data.

Execution plan (world = 1, default ``stream_mode="indep"``): one HIP graph replay runs
``steps_per_graph`` consecutive training steps, captured from two streams that stay independent for the
whole replay: the HDCE chain (its own gather, forward, backward, Adam) on one, the QSC chain (its own gather of
the same batch through a second device cursor, forward, backward, AdamW) on the other, joined once at the end
of the replay.  Almost every kernel of this model is latency-bound and fills a fraction of the 256 CUs, so the
QSC chain overlaps the HDCE chain, and the HDCE chain has no cross-queue edge (each one costs a queue
hand-over).  0.3997 / 0.4008 ms/step against 0.4104 / 0.4105 for ``"dagq"`` (the QSC branch forked after a
shared gather and joined before the HDCE update every step) on one box (profiles/r5_10_ab.txt); bit-identical
to the serial step.  (Round 3's independent plans shared the gather's classifier input across the streams --
the next step's gather could rewrite it under the QSC forward -- and were not reproducible: docs/CONCURRENCY.md.)
Per step:

  main : gather -> conv fwd x3 -> BN/ReLU apply (+ BN tail) -> FC fwd GEMM -> one-pass NMSE ->
         FC wgrad GEMM -> FC dgrad GEMM -> BN bwd reduce (+ loss finish) -> [wgrad|dgrad] L3 ->
         [wgrad|dgrad] L2 -> wgrad L1 -> slab sums (conv, BN, FC bias) -> (join) -> Adam (one launch over all
         HDCE parameters; also writes the bf16 FC shadow and the conv weights' MFMA B-fragment images
         for the NEXT step, and advances the batch cursor)
  qsc  : (after gather) QuantumNAT noise -> QSC fwd -> VQC fwd -> head -> VQC adjoint ->
         QSC bwd -> slabs -> AdamW

([wgrad|dgrad] = one launch running both independent gradients side by side.)

The HDCE and the QSC have separate NaN-guard flags (``skip[0]``, ``skip[1]``), so neither
optimizer waits for the other model's loss.
World > 1: five graphs around the gradient collectives (``_dp_run``): the FC gradient's collective
(reduce-scatter in the default ZeRO-1 plan, all-reduce otherwise) starts right after the forward +
FC weight gradient and is hidden by the FC data gradient, the conv backward and the QSC branch; the
FC update (Adam on this rank's shard + the bf16 weight all-gather, or Adam on all of it) runs on
its own stream and overlaps the next step's gather + conv forward.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Optional

import torch

from .. import _native as nat
from ..data.datasets import DMLStore, make_dml_stores
from ..models.estimators import QSC_P128
from ..ops.gather import StepGather
from ..knobs import KNOBS
from ..ops.optim import FlatParamSpace, make_optimizer
from ..ops.slabsum import SlabBatch
from ..parallel.dp import DistContext, GradBuckets
from ..utils.profiling import GraphedStep
from .engine import ClassifierStep, HDCEModel, HDCEStep
from .flagship_dp import DPPlan


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
    split_graphs: bool = False   # force the DP execution plan (5 graphs) even at world 1 (testing)
    stream_mode: str = "indep"   # serial | dagq | indep (see FlagshipTrainer.__init__)
    hdce_priority: bool = False  # (indep) capture on a high-priority stream: the HDCE chain's nodes keep that priority
    #                              over the QSC chain's (forked from a normal-priority stream) when both have work queued
    qsc_start: str = "step"      # (indep) "conv": each step's QSC chain waits for the HDCE conv forward (one HDCE ->
    #                              QSC edge, none on the HDCE chain), so the conv kernels have the chip to themselves
    tail_pack: bool = True       # pack the conv weights at the END of a step (not at the forward's head)
    fused_fc_adam: bool = False  # (world 1, GPU, bf16) the FC weight's Adam step in the weight-gradient GEMM's
    #                              epilogue (dW never written; bit-identical).  Off: 0.419-0.423 ms/step vs 0.412
    #                              separate (profiles/r3_04_fused_adam.txt) -- 256 one-per-CU workgroups stream
    #                              the Adam state far slower than the 2048-workgroup update kernel
    fc_adam_next: int = 0        # (world 1, indep) > 0: the FC weight's Adam on the "fc" stream after the step's other
    #                              Adam launch, on at most this many workgroups, overlapping the next step's gather + conv
    #                              forward; the next FC forward waits for it (the DP plan's overlap, at world 1).
    #                              2048 (the default launch size): 0.405 against 0.394 ms (profiles/r5_15_*)
    fc_adam_side: int = 0        # (world 1, dagq) > 0: the FC weight's Adam runs on the "fc" stream right after the FC
    #                              data gradient -- the last reader of the bf16 shadow it rewrites -- beside the conv
    #                              backward, on at most this many workgroups (so the conv kernels keep most CUs);
    #                              joined before the step's other Adam launch.  0: one Adam launch at the tail
    dp_plan: str = "zero"        # world > 1: "zero" = ZeRO-1 FC optimizer (reduce-scatter the FC gradient,
    #                              Adam on this rank's 1/world shard, all-gather the bf16 weight shadow) or
    #                              "allreduce" (all-reduce the FC gradient, every rank steps all of it)
    qsc_grid_bwd: int = 0        # QSC backward workgroups (0: at most 256, balanced to equal samples per wave)
    steps_per_graph: int = 1     # world 1: training steps captured per graph replay (run())
    lead_in: int = 1             # run(): the first lead_in steps replayed one step per graph -- a run that starts on
    #                              an idle GPU waits for its first graph's launch to be submitted, and a 1-step graph
    #                              is submitted in a fifth of a k-step one's time
    ramp: int = 4                # run(): after the lead-in, one ramp-step replay before the k-step ones.  A replay is
    #                              submitted by the host at ~0.08 ms per step while the GPU runs ~0.4 ms per step, and the
    #                              GPU starts a replay only once it is submitted: a k-step replay right behind a 1-step
    #                              one left the GPU idle for (0.08 k - 0.4) ms (0.35 ms of the driver's 20-step window,
    #                              BENCH_r04.json); behind a ramp-step replay every submission hides (0 = off)
    dp_one_graph: bool = False   # DP plan: capture the whole step -- its RCCL collectives included -- in ONE
    #                              graph (the 5-graph plan launches the collectives between graph replays and
    #                              pays a graph boundary at each; this one pays one per step but fences the
    #                              FC update at the end of the step instead of overlapping the next gather)
    dp_qsc: str = "g2"           # DP plan, where the QSC branch runs: "g2" = forked beside the conv backward (the most
    #                              work behind the FC gradient collective), "fwd" = forked right after the gather as in
    #                              the world-1 step, joined before the small bucket (shorter g2: wins where the FC
    #                              collective is short; one-graph plan only -- a fork cannot span two graphs);
    #                              "indep" (round 6) = the world-1 independent chains: the QSC chain with its own
    #                              gather, never joined inside the step, its gradients in a bucket of their own
    #                              all-reduced at the next step's start (DPPlan._dp_run_indep; all-reduce plan).
    #                              bench.py times them at the real world size.
    scaling: str = "weak"        # world > 1: "weak" = batch per stream on EVERY rank, each rank its own data; "strong" =
    #                              the reference's DataParallel semantics (R:144-148): ONE global batch of ``batch`` rows
    #                              per stream per step (same data and permutation on every rank) cut into world
    #                              contiguous parts of batch / world rows; the NMSE denominators are the global batch's
    #                              (gather.hip den_scale_kernel), so the ranks' losses are shares of one loss and the
    #                              HDCE gradients are SUMMED; per-rank BatchNorm (as DataParallel's replicas)
    seed: int = 0
    n_scenarios: int = 3
    n_users: int = 3


class FlagshipTrainer(DPPlan):
    def __init__(self, cfg: FlagshipConfig, ctx: DistContext, store: Optional[DMLStore] = None):
        """``store``: share another trainer's HBM-resident dataset (same data_len / pilots / SNR / seed)."""
        self.cfg, self.ctx = cfg, ctx
        dev = ctx.device
        if cfg.scaling not in ("weak", "strong"):
            raise ValueError(f"scaling {cfg.scaling!r}")
        self.strong = cfg.scaling == "strong" and ctx.world > 1
        if self.strong and cfg.batch % ctx.world:
            raise ValueError(f"scaling 'strong': batch {cfg.batch} is not split evenly over {ctx.world} ranks")
        if store is None:
            # (strong: every rank holds the same data -- its part of each global batch comes from it)
            store, _ = make_dml_stores(cfg.data_len, cfg.pilot_num, cfg.snr_db, 0.9, dev, data_dir=None, synthetic=True,
                                       base_seed=cfg.seed + (0 if self.strong else 1000 * ctx.rank),
                                       n_scenarios=cfg.n_scenarios, n_users=cfg.n_users)
        self.store = store
        self.E, self.U = cfg.n_scenarios, cfg.n_users
        self.Bg = cfg.batch                                           # rows per stream of one step's (global) batch
        self.B = cfg.batch // ctx.world if self.strong else cfg.batch   # this rank's rows per stream
        # HDCE gradient scale: weak -- the mean of the ranks' losses; strong -- shares of ONE loss, summed
        self._hgs = 1.0 if self.strong else 1.0 / ctx.world
        self.S = self.E * self.U
        # --- models (weights broadcast from rank 0 once; then resident)
        torch.manual_seed(cfg.seed)
        dp = ctx.world > 1 or cfg.split_graphs
        if cfg.dp_plan not in ("zero", "allreduce"):
            raise ValueError(f"dp_plan {cfg.dp_plan!r}")
        if cfg.dp_qsc not in ("g2", "fwd", "indep") or (cfg.dp_qsc in ("fwd", "indep") and not cfg.dp_one_graph):
            raise ValueError(f"dp_qsc {cfg.dp_qsc!r} (\"fwd\" / \"indep\" need dp_one_graph)")
        if cfg.dp_qsc == "indep" and cfg.dp_plan != "allreduce":
            raise ValueError("dp_qsc 'indep' runs on the all-reduce plan (ZeRO's HDCE NaN flag rides in the QSC bucket)")
        # ZeRO-1 plan (see _dp_run); not with the fp8 estimator (its weight scale is a max over the
        # whole FC weight, which a sharded update would have to all-reduce)
        self.zero = dp and cfg.dp_plan == "zero" and cfg.dtype != "fp8"
        # all-reduce plan: the HDCE NaN flag lives in a scratch slot right after the FC gradient, so it
        # travels in the FC all-reduce (one collective less ahead of it); ZeRO plan: in the small bucket
        # (every rank needs the summed flag, a reduce-scatter leaves it on one rank only)
        self.flag_in_fc = dp and not self.zero
        # DP: the QSC space lives IN FRONT of the HDCE space in one allocation, and the NaN flags in its trailing
        # scratch (QSC flag at +0, ZeRO's HDCE flag one 128-byte line later), so the small bucket -- QSC grads,
        # flags, conv/BN grads -- is ONE contiguous range: all-reduced in place, no coalescing / scatter-back
        # copies on the step's critical path.  (Sized on the meta device: no RNG draw, init order unchanged.)
        qargs = (cfg.n_qubits, cfg.n_layers, cfg.n_classes, cfg.use_quantumnat, cfg.use_gradient_pruning,
                 cfg.pilot_num)
        q_extra = 64 if dp else 0
        nq = 0
        if dp:
            with torch.device("meta"):
                nq = FlatParamSpace.size_of(list(QSC_P128(*qargs).named_parameters()), extra=q_extra)
        self.hdce = HDCEModel(cfg.pilot_num, dev, cfg.dtype, cfg.n_scenarios, grad_extra=1 if self.flag_in_fc else 0,
                              fc_pad_multiple=ctx.world if self.zero else 1, front=nq)
        self.qsc = QSC_P128(*qargs).to(dev)
        self.qspace = FlatParamSpace(list(self.qsc.named_parameters()), dev, extra=q_extra,
                                     storage=self.hdce.space.front_views)
        ctx.broadcast_(self.hdce.space.flat)
        ctx.broadcast_(self.qspace.flat)
        self.hopt = make_optimizer(self.hdce.space, "adam", cfg.lr)
        sp = self.hdce.space
        n_conv = sp.offsets[sp.names.index("CE.FC.weight")]
        # part 0: conv + BN params, part 1: FC -- for the plans that step them apart (the DP plan, the FC
        # Adam side branch); the world-1 chain steps the whole space in ONE launch
        # ZeRO: parts 1..world = the FC region [n_conv, end) in equal shards; this rank steps 1 + rank
        self.fc_region = (n_conv, sp.numel)
        self.shard_len = (sp.numel - n_conv) // ctx.world
        if self.zero:
            self.hopt.partition([n_conv + i * self.shard_len for i in range(ctx.world)])
        elif dp:
            self.hopt.partition([n_conv])
        # after the broadcast: the shadow starts in sync
        self.hdce.attach_fc_shadow(self.hopt, to_end=self.zero)
        self.qopt = make_optimizer(self.qspace, "adamw", cfg.lr, weight_decay=cfg.qsc_weight_decay,
                                   prune_thr=0.1 if cfg.use_gradient_pruning else 0.0)
        # the NaN flags in the spaces' trailing scratch (below) are read by the update kernels while they run:
        # neither optimizer steps them (a step writes grad_scale-d / pruned gradients back in place)
        if dp:
            self.qopt.limit(self.qspace.extra_off)
        if self.flag_in_fc:
            self.hopt.limit(sp.extra_off)
        self.hstep = HDCEStep(self.hdce, self.U, self.B)
        self.hstep.bias_via_conv_slabs = ctx.world == 1 and not cfg.split_graphs
        # NaN guards: the NMSE kernel sets skip[0] (HDCE), the QSC head skip[1]; they travel in the
        # small bucket so every rank sees the same (summed) flags and skips -- or steps -- in lockstep
        self.skip = torch.zeros(2, 64, device=dev, dtype=torch.float32)   # (own cache line per flag)
        self.qskip = self.skip[1, 0:1]
        self.hskip = sp.grad[sp.extra_off:sp.extra_off + 1] if self.flag_in_fc else self.skip[0, 0:1]
        if dp:
            qe = self.qspace.extra_off
            self.qskip = self.qspace.grad[qe:qe + 1]
            if self.zero:
                self.hskip = self.qspace.grad[qe + 32:qe + 33]
        self.hstep.nmse.skip = self.hskip
        # (QSC backward workgroups: at most 256, balanced to the same samples per wave -- 192 at 2304 samples --
        # unless set; fewer measured slower, profiles/r2_20_variants.md, r6_06_qsc_grid_fp8_ab.txt)
        gb = cfg.qsc_grid_bwd or 256
        self.cstep = ClassifierStep(self.qsc, self.S, space=self.qspace, batch_total=self.S * self.B,
                                    skip=self.qskip, hip_kw={"grid_bwd": gb, "balance_bwd": not cfg.qsc_grid_bwd})
        self.cstep.skip_add = False
        self.cstep.writes_grads = self.cstep.hip is not None
        # buckets (see _dp_run): "fc" = 33.6 MB FC grads (in place; + the HDCE NaN flag in the all-reduce plan),
        # "small" = QSC grads + NaN flags + conv/BN grads, one contiguous range in place (DP; see above)
        bk = {"fc": [sp.grad[n_conv:]], "small": [sp.grad[:n_conv], self.qspace.grad, self.qskip]}
        if dp:
            bk["small"] = [sp.grad_base[:nq + n_conv]]
            if cfg.dp_qsc == "indep":   # (the QSC chain's own bucket: its gradients + NaN flag, all-reduced apart)
                bk["small"], bk["q"] = [sp.grad_base[nq:nq + n_conv]], [sp.grad_base[:nq]]
            if self.zero:
                del bk["fc"]   # (its reduce-scatter is launched on the region directly)
        else:
            bk["skip"] = [self.skip[0, 0:1]]
        self.buckets = GradBuckets(ctx, bk)
        self.gat = StepGather(self.E, self.U, self.B, self.hdce.H, self.hdce.W, dev, with_classifier=True)
        if dev.type == "cuda" and self.hstep.hip:   # per-row label powers ride along with the gather
            nm = self.hstep.nmse
            self.gat.rowpow = (nm._row_powers(self.store.Hlabel), nm._row_powers(self.store.Hperf))
        if self.strong:
            self.gat.set_part(ctx.rank * self.B, self.Bg)
            if dev.type == "cuda" and not self.hstep.hip:
                raise ValueError("scaling 'strong' on a GPU needs the HIP HDCE step (its NMSE reads scaled row powers)")
            if dev.type != "cuda":   # (the torch NMSE takes the global denominators directly)
                self.hstep.nmse.den_global = self.gat.den_global
        # batch selection on the device: the gather kernels read perm[cur : cur + B] and advance cur
        # themselves (cur[0]: HDCE / whole-step gather, cur[1]: the QSC graph's own gather); the host
        # only tracks the epoch position to regenerate perm in place when it runs out
        self.perm = torch.randperm(self.store.n, device=dev)
        if self.strong:
            ctx.broadcast_(self.perm)   # (one permutation: the ranks take parts of the same global batches)
        # (one 256-byte row each: the HDCE and QSC chains run concurrently and update their own
        # cursor / arrival counter, so the two never share a cache line)
        self.cur = torch.zeros(2, 64, dtype=torch.int32, device=dev)
        self.cur_done = torch.zeros(2, 64, dtype=torch.int32, device=dev)
        self.cursor = 0   # host mirror of the device cursors (position of the NEXT batch)
        # the loss kernels' own static buffers double as the step's loss outputs (no per-step copies)
        self.hloss = self.hstep.nmse.loss
        self.qloss = self.cstep.hip.loss if self.cstep.hip is not None else torch.zeros(1, device=dev)
        self.labels = self.store.scen.repeat_interleave(self.B)
        self.qslabs = SlabBatch()
        graphs = cfg.hip_graphs and dev.type == "cuda"
        # side streams (GPU).  stream_mode:
        #   serial : one stream, one chain
        #   dagq   : ONE graph, the QSC branch forked after the gather and joined at the end of the step; the
        #            HDCE a single chain.  (The DP plan also forks the FC update onto the "fc" stream.)
        #   indep  : (world 1) the QSC chain with its own gather, independent of the HDCE chain for the whole
        #            k-step replay (_indep_step); world > 1 runs the DP plan as with dagq
        # (a HIP graph's executor maps parallel branches onto its own pool of queues and every edge that
        # crosses queues costs a barrier packet, so fewer, longer branches win.  Measured and removed in round 3
        # (docs/CONCURRENCY.md): HDCE side branches (FC wgrad / conv wgrads / FC Adam on their own streams),
        # QSC and HDCE chains independent across step boundaries (1-1.5% faster, not bit-reproducible),
        # CU-masked streams for the two chains (ops/streams.py: every partition slower), and the DP plan's
        # QSC branch split around the HDCE forward.)
        mode = cfg.stream_mode
        if mode not in ("serial", "dagq", "indep"):
            raise ValueError(f"stream_mode {mode!r}")
        self.streams = None
        if dev.type == "cuda" and mode != "serial" and self.hstep.hip and self.cstep.hip is not None:
            self.streams = {k: torch.cuda.Stream(dev) for k in ("qsc", "fc")}
        else:
            mode = "serial"
        self.mode = mode
        # the FC weight's Adam in the weight-gradient GEMM's epilogue (world 1: no gradient collective between)
        self.fused_adam = bool(cfg.fused_fc_adam and dev.type == "cuda" and ctx.world == 1 and not cfg.split_graphs
                               and self.hstep.hip and "wgrad" in self.hstep.hand_gemm and not self.hdce.fp8
                               and cfg.dtype == "bf16" and len(self.hopt.bounds) == 1
                               and self.S * self.B % 64 == 0)   # (the hand weight-gradient GEMM's M tiling)
        if self.fused_adam:
            lo = sp.offsets[sp.names.index("CE.FC.weight")]
            slot = self.hopt.fuse_range(lo, lo + self.hdce.fc_w.numel())
            self.hstep.fused_adam = {"opt": self.hopt, "lo": lo, "slot": slot, "skip": self.hskip}
            # the fused update reads this step's NaN flag: the loss finish (which sets it) runs right after the
            # loss pass, not deferred into the conv backward
            self.hstep.defer_loss = False
        self.fc_adam_side = bool(cfg.fc_adam_side > 0 and not self.fused_adam and self.streams is not None
                                 and mode == "dagq"
                                 and cfg.dtype == "bf16" and self.hdce.fc_shadow is not None
                                 and ctx.world == 1 and not cfg.split_graphs and len(self.hopt.bounds) == 1)
        if self.fc_adam_side:
            lo = sp.offsets[sp.names.index("CE.FC.weight")]
            self.hopt.fuse_range(lo, lo + self.hdce.fc_w.numel())
            self.hstep.after_dgrad = self._fc_adam_fork
        self.fc_adam_next = bool(cfg.fc_adam_next > 0 and not self.fused_adam and not self.fc_adam_side
                                 and self.streams is not None and mode == "indep" and self.hstep.hip
                                 and cfg.dtype == "bf16" and self.hdce.fc_shadow is not None
                                 and ctx.world == 1 and not cfg.split_graphs and len(self.hopt.bounds) == 1)
        if self.fc_adam_next:
            lo = sp.offsets[sp.names.index("CE.FC.weight")]
            self.hopt.fuse_range(lo, lo + self.hdce.fc_w.numel())
        self._fc_pending = False   # (fc_adam_next) an FC update forked in this replay that the next FC forward awaits
        # (world 1) the HDCE update sums the step's gradient slabs itself: the slab launch leaves the chain
        self.adam_slabs = bool(KNOBS.adam_slabs and self.hstep.hip and ctx.world == 1 and not cfg.split_graphs
                               and self.hstep.writes_grads and self.hopt.kind in ("adam", "adamw")
                               and len(self.hopt.bounds) == 1 and not self.fused_adam)
        self.hstep.defer_slabs = self.adam_slabs
        # end-of-step weight pack (GPU fused path)
        self.tail_pack = bool(self.hstep.hip and cfg.tail_pack)
        if self.tail_pack:
            self.hstep.conv.pack_at_tail = True
            self._tail_pack_launch(advance=False)   # the first step's images
        self._use_graphs = graphs
        self._phases = None   # (phase_times) per-step dicts of HIP events
        self._stamps = None   # (phase_times, one-graph plan) (device clock buffer, {phase: slot}) while capturing
        self._prime_fp8()
        self._graph_sets = {}            # steps per replay -> list of GraphedStep
        self.graphs = self._graphs_for(1)

    def _prime_fp8(self) -> None:
        """(fp8 estimator) seed the loss gradient's delayed e4m3 scale before the first step
        (HDCEStep.prime_fp8_dy).  The primed slot is part of mutable_state(), so a capture(preserve=True)
        restores it primed."""
        def fwd():
            self._gather(classifier=False)
            self._hdce_forward()
            return self.hstep
        if self.hstep.prime_fp8_dy(fwd, self.mutable_state() + [self.cur], self.ctx) and self.tail_pack:
            self._tail_pack_launch(advance=False)   # (the packed conv images of the restored weights)

    def _graphs_for(self, k: int):
        """The graph set that runs ``k`` consecutive training steps per replay (world 1; the DP plan is
        always one step).  Every step of a replay gathers its own batch through the device cursor, so a
        k-step replay IS k training steps: the graph boundary is paid once per k steps."""
        if k in self._graph_sets:
            return self._graph_sets[k]
        graphs, cfg, mode = self._use_graphs, self.cfg, self.mode

        def rep(fn):
            def body():
                for _ in range(k):
                    fn()
            return body

        if self.ctx.world == 1 and not cfg.split_graphs and mode == "indep":
            # the QSC and HDCE chains independent for the whole k-step replay (see _indep_step): one join at its end
            def body():
                self._fc_pending = False
                for i in range(k):
                    self._indep_step(first=i == 0)
                self._join(("qsc", "fc") if self._fc_pending else ("qsc",))
                self._fc_pending = False
            cs = torch.cuda.Stream(self.ctx.device, priority=-1) if (cfg.hdce_priority and graphs) else None
            gs = [GraphedStep(body, enabled=graphs, capture_stream=cs)]
        elif self.ctx.world == 1 and not cfg.split_graphs:
            # one graph: gather, both forwards, NMSE, both backwards, the optimizers
            gs = [GraphedStep(rep(self._step_body), enabled=graphs)]
        else:
            if cfg.dp_one_graph and graphs:
                # the collectives are captured too: RCCL kernels become graph nodes on the PG's stream,
                # ordered by the captured event edges exactly as the eager plan orders them.  k steps per
                # replay: step i's FC update (fc stream) overlaps step i + 1's gather + conv forward
                def body():
                    for i in range(k):
                        if cfg.dp_qsc == "indep" and self.streams is not None:
                            self._dp_run_indep(fence=i == k - 1, first=i == 0)
                        else:
                            self._dp_run(self._dp_g1a, self._dp_g1b, self._dp_g2, self._dp_gf, self._dp_gr,
                                         fence=i == k - 1, first=i == 0)
                gs = [GraphedStep(body, enabled=graphs, guards=(self.buckets.assert_quiescent,))]
                self._graph_sets[k] = gs
                return gs
            if k != 1:
                raise ValueError("multi-step graphs are a world-1 plan (and the one-graph DP plan's)")
            # five graphs around the gradient collectives (see _dp_run); one memory pool is safe: the
            # graphs that replay concurrently (gf on the fc stream beside gr / the next g1a on main)
            # allocate nothing
            pool = torch.cuda.graph_pool_handle() if graphs else None
            gs = [GraphedStep(f, enabled=graphs, pool=pool, guards=(self.buckets.assert_quiescent,))
                  for f in (self._dp_g1a, self._dp_g1b, self._dp_g2, self._dp_gf, self._dp_gr)]
        self._graph_sets[k] = gs
        return gs

    # -- phases ---------------------------------------------------------------------------
    def _fork(self, s) -> "torch.cuda.StreamContext":
        s.wait_stream(torch.cuda.current_stream(self.ctx.device))
        return torch.cuda.stream(s)

    def _join(self, names=("qsc", "fc")) -> None:
        cur = torch.cuda.current_stream(self.ctx.device)
        for n in names:
            cur.wait_stream(self.streams[n])

    def _gather(self, hdce: bool = True, classifier: bool = True) -> None:
        # the fused GPU kernels WRITE every gradient (one producer per element): no zero_grad fills
        if hdce and not self.hstep.writes_grads:
            self.hdce.space.zero_grad()
        if classifier and not self.cstep.writes_grads:
            self.qspace.zero_grad()
        # one launch: conv input, classifier input, label rows; batch = perm[cur : cur + B].  With the
        # end-of-step weight pack (tail_pack) the pack advances cur[0]; else the gather itself does
        k = 0 if hdce else 1
        advance = not (self.tail_pack and k == 0)
        self.gat.from_cursor(self.store, self.perm, self.cur[k, 0:1], self.cur_done[k, 0:1] if advance else None,
                             hdce=hdce, classifier=classifier)

    def _adam_pack(self):
        """(tail_pack) the HDCE update writes the conv weight images and advances the batch cursor
        itself (no separate pack launch after it)."""
        if not self.tail_pack:
            return None
        conv, flat, cur = self.hstep.conv, self.hdce.space.flat, self.cur[0, 0:1]
        return lambda lo, hi: conv.pack_scatter(flat, lo, hi, cursor=cur, cursor_inc=self.Bg)

    def _tail_pack_launch(self, advance: bool = True) -> None:
        """Pack the (just updated) conv weights into the MFMA B-fragment images the next forward reads,
        and advance the batch cursor -- one launch at the end of the step."""
        self.hstep.conv.pack_weights(nat.stream_ptr(self.ctx.device), cursor=self.cur[0, 0:1] if advance else None,
                                     cursor_inc=self.Bg if advance else 0)

    def _fc_adam_fork(self) -> None:
        """(fc_adam_side) the FC weight's Adam on the fc stream, after the FC data gradient (its last reader of the
        shadow) and the loss pass (its NaN flag); the step joins the stream before its other Adam launch."""
        with self._fork(self.streams["fc"]):
            self.hopt.step_fused(grad_scale=1.0, skip=self.hskip, max_grid=self.cfg.fc_adam_side)

    def _qsc_branch(self, with_opt: bool) -> None:
        """The QSC step (+ AdamW with ``with_opt``)."""
        q = self.cstep(self.gat.xq, self.labels, slabs=self.qslabs if self.cstep.writes_grads else None)
        if self.cstep.writes_grads:
            self.qslabs.launch(accumulate=False, stream=nat.stream_ptr(self.ctx.device))
        if q is not self.qloss:
            self.qloss.copy_(q)
        if with_opt:
            self.qopt.step(grad_scale=1.0 / self.ctx.world, skip=self.qskip)

    def _hdce_forward(self) -> None:
        loss = self.hstep.forward_fc_gathered(self.gat, self.store)
        if loss is not self.hloss:
            self.hloss.copy_(loss)

    def _hdce_graph(self) -> None:
        """HDCE forward + backward + Adam (world 1): one Adam launch over the whole space, which also packs
        the next step's conv weight images and advances the batch cursor (tail_pack)."""
        self._hdce_forward()
        self._hdce_backward_update()

    def _hdce_backward_update(self) -> None:
        """conv/BN backward + the one Adam launch over the whole HDCE space (+ the conv weight images)."""
        self.hstep.backward_conv()
        self._hdce_update()

    def _hdce_update(self) -> None:
        pk = self._adam_pack()
        sl = self.hstep.take_slabs() if self.adam_slabs else None
        self.hopt.step(grad_scale=1.0, skip=self.hskip, pack=pk, slabs=sl)
        if self.tail_pack and pk is None:
            self._tail_pack_launch()

    def _step_body(self) -> None:
        if self.mode == "dagq":
            # the QSC branch forks right after the batch gather: its latency-bound kernels share the GPU with
            # the HDCE chain's, and it joins BEFORE the HDCE update (the QSC branch has long finished by then).
            # The update is then the chain's last node with a single parent on its own queue, and the next
            # step's gather follows it there; with the join after the update, the graph executor placed the
            # gather on the QSC queue and every step paid two cross-queue hops (update -> gather -> conv
            # forward, ~33 us idle: profiles/r3_23_step_timeline.md).  0.4176-0.4182 vs 0.4203-0.4223 ms/step
            # (profiles/r4_08_plan_probe.txt).  (Measured alternatives, round 4, docs/CONCURRENCY.md: the HDCE
            # chain captured first, the QSC branch gathering its own batch, the QSC step split around the FC
            # GEMMs, the FC update on the QSC stream -- all slower.)
            self._gather()
            with self._fork(self.streams["qsc"]):
                self._qsc_branch(with_opt=True)
            self._hdce_forward()
            self.hstep.backward_conv()
            self._join(("qsc", "fc") if self.fc_adam_side else ("qsc",))
            self._hdce_update()
            return
        self._dp_run(self._dp_g1a, self._dp_g1b, self._dp_g2, self._dp_gf, self._dp_gr)

    def _indep_step(self, first: bool) -> None:
        """(stream_mode "indep", world 1) one training step with the QSC chain fully independent of the HDCE
        chain: the QSC branch gathers its own half of the batch (the same permutation through its own cursor,
        cur[1], so both models see the same samples) on its own stream and is never joined inside the replay, so
        the HDCE chain -- gather, forward, backward, Adam -- has no cross-queue edge at all (the dagq step pays
        two queue hand-overs per step at its join, ~14 us).  The classifier input is written and read on the qsc
        stream only (round 3's independent plans shared the gather's output across the streams: that race is why
        they were not reproducible).  ``first``: the replay's first step orders the qsc stream after this step's
        first node (a branch forked before any node would be a root of the graph)."""
        self._gather(classifier=False)
        q = self.streams["qsc"]
        after_conv = (self.cfg.qsc_start == "conv" or self.fc_adam_next) and self.hstep.hip
        if after_conv:
            self.hstep.forward_conv_gathered(self.gat)
            if self._fc_pending:   # (fc_adam_next) the FC forward reads the weights the previous step's update wrote
                torch.cuda.current_stream(self.ctx.device).wait_stream(self.streams["fc"])
        if first or (after_conv and self.cfg.qsc_start == "conv"):
            q.wait_stream(torch.cuda.current_stream(self.ctx.device))
        with torch.cuda.stream(q):
            self._gather(hdce=False, classifier=True)
            self._qsc_branch(with_opt=True)
        if after_conv:
            loss = self.hstep.forward_fc_after_conv(self.store)
            if loss is not self.hloss:
                self.hloss.copy_(loss)
        else:
            self._hdce_forward()
        self.hstep.backward_conv()
        self._hdce_update()
        if self.fc_adam_next:
            with self._fork(self.streams["fc"]):
                self.hopt.step_fused(grad_scale=1.0, skip=self.hskip, max_grid=self.cfg.fc_adam_next)
            self._fc_pending = True

    def skip_flags(self) -> torch.Tensor:
        """(2,) the HDCE and QSC NaN-guard flags of the last step (after the all-reduce: summed)."""
        return torch.cat([self.hskip, self.qskip])

    def mutable_state(self):
        """Every tensor a step updates in place (weights, optimizer moments/counters, BN running
        statistics, the fp8 scales, the QuantumNAT RNG counter)."""
        ts = [self.hdce.space.flat, self.qspace.flat, self.hopt.step_t, self.qopt.step_t]
        for o in (self.hopt, self.qopt):
            ts += [o.m, o.v] if o.kind != "sgd" else [o.buf]
        ts += list(self.hdce.run_mean) + list(self.hdce.run_var) + [self.hdce._nbt]
        if self.hdce.fc_shadow is not None:
            ts.append(self.hdce.fc_shadow)
        if self.hopt.shadow8 is not None:
            ts.append(self.hopt.shadow8)
        if getattr(self.hdce, "fp8_scales", None) is not None:
            f8 = self.hdce.fp8_scales
            ts += [f8.scale, f8.qs, f8.amax]
        if self.cstep.hip is not None:
            ts.append(self.cstep.hip.noise_ctr)
        return ts

    def capture(self, preserve: bool = True, k: int = 1) -> None:
        """Capture the ``k``-step graph set now.  Capturing runs warm-up steps; with ``preserve`` the
        model/optimizer state is restored afterwards, so the first real step is step 1."""
        self._capture_set(self._graphs_for(k), k, preserve)

    def _capture_set(self, gs, k: int, preserve: bool = True) -> None:
        """Capture the graphs of ``gs`` (``k`` steps per replay) that are not captured yet."""
        if not any(g.enabled and g.graph is None for g in gs):
            return
        # the warm-up runs inside capture advance the device cursors: make room, restore them after
        if self.cursor + (GraphedStep.WARMUP + 1) * k * self.Bg > self.store.n:
            self._new_epoch()
        if self.cursor + (GraphedStep.WARMUP + 1) * k * self.Bg > self.store.n:
            raise ValueError(f"{k} steps per graph need more than the {self.store.n} samples per stream")
        cur = self.cur.clone()
        saved = [t.clone() for t in self.mutable_state()] if preserve else None
        for g in gs:
            if g.enabled and g.graph is None:
                g.capture()
        if saved is not None:
            for t, c in zip(self.mutable_state(), saved):
                t.copy_(c)
        self.cur.copy_(cur)
        if self.tail_pack:   # (the packed images are derived from the weights: rebuild them)
            self._tail_pack_launch(advance=False)

    @property
    def graphed(self) -> GraphedStep:
        return self.graphs[0]

    def _new_epoch(self) -> None:
        # in place: the graphs hold its address; the previous replays were joined on this stream
        torch.randperm(self.store.n, device=self.ctx.device, out=self.perm)
        if self.strong:
            self.ctx.broadcast_(self.perm)
        self.cur.zero_()
        self.cursor = 0

    def next_batch(self, k: int = 1) -> None:
        """Advance the host mirror of the batch cursor by ``k`` batches; when the permutation cannot
        hold them, draw a new one and re-arm the device cursors (the short tail is dropped)."""
        if self.cursor + k * self.Bg > self.store.n:
            self._new_epoch()
        self.cursor += k * self.Bg

    def step(self) -> None:
        """One training step."""
        self._replay(1)

    def _k(self) -> int:
        one = (self.ctx.world == 1 and not self.cfg.split_graphs) or (self.cfg.dp_one_graph and self._use_graphs)
        if not one:
            return 1
        # (a capture runs WARMUP + 1 passes of the k steps inside one permutation of the stream: large batches --
        # P256 x 1024 samples per stream -- get fewer steps per replay)
        fit = self.store.n // ((GraphedStep.WARMUP + 1) * self.Bg)
        return max(1, min(self.cfg.steps_per_graph, fit))

    def _reps(self, n: int):
        """Steps per replay of ``run(n)``: lead_in single steps, one ``ramp``-step replay, then k-step replays; a
        remainder r rides in the LAST of them as one (k + r)-step graph where the dataset holds that capture
        (every replay boundary drains both chains and re-fills them, ~30 us: profiles/r5_46_bench*.json), else it
        is one replay of its own.  Each replay is submitted while the previous one runs, so the ramp keeps every
        submission behind GPU work (FlagshipConfig.ramp).  The driver's 20-step window is [1, 4, 15]: three
        boundaries instead of [1, 4, 10, 5]'s four."""
        k = self._k()
        if k == 1:
            return [1] * n
        head = [1] * max(0, self.cfg.lead_in)
        if head and 1 < self.cfg.ramp < k:
            head.append(self.cfg.ramp)
        fit = self.store.n // ((GraphedStep.WARMUP + 1) * self.Bg)   # (what _capture_set can hold: see _k)
        sub, g = getattr(self, "_sub_est", None), getattr(self, "_g_est", None)
        if head and sub and g and g > sub[1]:
            return self._reps_calibrated(n, k, fit, sub, g)
        reps, rem = [], n
        for r in head:
            if rem == 0:
                break
            reps.append(min(r, rem))
            rem -= reps[-1]
        body, tail = [k] * (rem // k), rem % k
        if tail and body and k + tail <= fit:
            body[-1] += tail
            tail = 0
        return reps + body + ([tail] if tail else [])

    BOUNDARY_S = 30e-6   # what a replay boundary costs the GPU (both chains drain and refill): bench windows, r5-r6
    SUBMIT_MARGIN = 1.2  # the host's submission pace varies between replays

    def _reps_calibrated(self, n: int, k: int, fit: int, sub, g: float):
        """The replay plan from measured rates (``calibrate``): submitting an r-step replay takes the host
        ``a + c r`` seconds (``sub`` = (a, c)), the GPU runs g seconds per step and b per replay boundary.  A replay
        starts on the GPU only once its submission is complete, so after the 1-step lead-in every replay is as long
        as the GPU work queued ahead of it can hide: its submission must end before the GPU finishes the replays
        before it -- the sizes grow roughly geometrically at ratio g / c -- capped at ``fit`` steps per graph.  (A fixed
        [1, 4, 15] left the GPU idle 0.3 ms behind the 15-step submission on a slow-host box, 0.4162 against 0.3956
        ms/step: profiles/r6_01_bench20*.json.)"""
        b = self.BOUNDARY_S
        a, c = (self.SUBMIT_MARGIN * v for v in sub)
        reps = [1]
        host = a + c           # the lead-in's submission ends
        gpu = host + g + b     # ... and the GPU finishes it
        S = 1
        while S < n:
            allowed = int((gpu - host - a) / c) if c > 0 else fit
            r = max(1, min(allowed, fit, n - S))
            if 0 < n - S - r < max(2, k // 2) and n - S <= fit:   # (no tiny tail replay)
                r = n - S
            host += a + c * r
            gpu = max(gpu, host) + g * r + b
            reps.append(r)
            S += r
        return reps

    def note_submission(self, k: int, seconds: float) -> None:
        """(host submission rate) seconds the host spent submitting a k-step replay (kept: the last 64)."""
        subs = getattr(self, "_subs", None)
        if subs is None:
            subs = self._subs = []
        subs.append((k, seconds))
        del subs[:-64]

    @staticmethod
    def _fit_submission(subs):
        """(a, c): least-squares fit of submit seconds = a + c k over the noted replays (fixed cost + per step)."""
        if not subs:
            return 0.0, 0.1e-3
        ks = sorted({k for k, _ in subs})
        if len(ks) < 2:
            return 0.0, sorted(t / k for k, t in subs)[len(subs) // 2]
        n = len(subs)
        mk = sum(k for k, _ in subs) / n
        mt = sum(t for _, t in subs) / n
        var = sum((k - mk) ** 2 for k, _ in subs)
        c = sum((k - mk) * (t - mt) for k, t in subs) / var
        a = mt - c * mk
        if c <= 0:
            return 0.0, mt / mk
        return max(a, 0.0), c

    def calibrate(self, gpu_s_per_step: float) -> None:
        """Rates for the replay plan (``_reps_calibrated``): the GPU's seconds per step (e.g. a synchronised run's wall
        time per step, every graph set of it captured beforehand) and the host's submission cost (fitted over the
        replays submitted so far).  World > 1: the slowest rank's rates, so every rank runs the same plan."""
        a, c = self._fit_submission(getattr(self, "_subs", []))
        g = float(gpu_s_per_step)
        if self.ctx.world > 1:
            a, c, g = self.ctx.max_vector([a, c, g])
        self._sub_est, self._g_est = (a, c), g

    def prepare(self, n: int) -> None:
        """Capture every graph set ``run(n)`` will replay (keeps capture out of a timed region)."""
        for kk in sorted(set(self._reps(n)), reverse=True):
            self.capture(preserve=True, k=kk)

    def run(self, n: int) -> None:
        """``n`` training steps, ``cfg.steps_per_graph`` per graph replay (lead_in single steps first, the
        remainder as one shorter graph)."""
        reps = self._reps(n)
        for i, kk in enumerate(reps):   # (DP plan: consecutive steps overlap; the last one is fenced)
            self._replay(kk, fence=i == len(reps) - 1)

    def _replay(self, k: int, fence: bool = True) -> None:
        if getattr(self, "_closed", False):
            raise RuntimeError("FlagshipTrainer used after close()")
        gs = self._graphs_for(k)
        if any(g.enabled and g.graph is None for g in gs):
            # (preserve: the capture warm-ups run optimizer steps on rank-local gradients; restoring
            # the state keeps the ranks bit-identical)
            self.capture(preserve=True, k=k)
        self.next_batch(k)
        self.steps_done = getattr(self, "steps_done", 0) + k   # (optimizer steps applied: capture warm-ups excluded)
        if len(gs) == 1:
            t0 = time.perf_counter()
            gs[0]()
            self.note_submission(k, time.perf_counter() - t0)
            return
        self._dp_run(*gs, fence=fence)

    @property
    def samples_per_step(self) -> int:
        return self.S * self.B

    def close(self) -> None:
        """Retire every captured graph set now (GraphedStep.close: the executables are parked and destroyed at exit
        -- utils/profiling.py GRAPH_RELEASE -- never by whichever garbage collection reaches them, possibly in the
        middle of another trainer's capture or replay).  Idempotent; the trainer cannot step afterwards."""
        for gs in list(getattr(self, "_graph_sets", {}).values()):
            for g in gs:
                g.close()
        self._graph_sets = {}
        self.graphs = []
        self._closed = True
