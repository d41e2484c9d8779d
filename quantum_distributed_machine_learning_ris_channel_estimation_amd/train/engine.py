"""Fused training engines for the HDCE estimator and the scenario classifiers.

Reference hot loops (Runner_P128_QuantumNAT_onchipQNN.py):
  * HDCE (R:181-204): for each of 9 (scenario, user) streams, pack on the host, H2D,
    run Conv[sid] then the shared CE under DataParallel (which re-broadcasts the 32 MiB
    FC weight and reduces its gradient to GPU0 on EVERY call), NMSE loss / 9, and a
    separate ``backward()`` per stream; then step 4 Adam optimizers.
  * QSC (R:335-370): 9 serial forwards of the hybrid classifier, one backward, pruning,
    AdamW.

MI355X design implemented here:
  * the dataset is HBM-resident (data/datasets.DMLStore); a step gathers its rows on
    the device -- no host packing, no H2D;
  * all 9 streams are ONE step.  The three scenario experts run as one grouped
    convolution: the expert index is folded into the channel axis (input
    (3*B, 3*2, H, W), groups=3), so one kernel per layer serves all experts and the
    per-expert activations land, already flattened C-major, as rows of a single
    (9*B, 4096) FC operand (rows ordered user, batch, expert);
  * BatchNorm is "ghost" BN over each 256-sample stream batch -- exactly the
    statistics the reference's per-stream Conv calls see (R:194), including three
    sequential momentum updates of each expert's running stats per step;
  * the FC GEMM runs in bf16 with fp32 accumulation; the per-stream NMSE and its
    gradient come from the fused kernels in ops/nmse.py;
  * backward is split explicitly at the FC input: FC grads (32 MiB) are complete
    first, so data-parallel all-reduce of that bucket overlaps the conv backward;
  * parameters live in FlatParamSpaces; the optimizer step is one kernel.
"""
from __future__ import annotations



from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native as nat
from ..knobs import KNOBS
from ..models.estimators import Conv_P128, FC_P128, QSC_P128, SC_P128, pilot_grid
from ..ops.nmse import StreamNMSE
from ..ops.optim import ALIGN, FlatParamSpace

CONV_PARAM_ORDER = ["cnn.0.weight", "cnn.1.weight", "cnn.1.bias", "cnn.3.weight", "cnn.4.weight", "cnn.4.bias",
                    "cnn.6.weight", "cnn.7.weight", "cnn.7.bias"]
BN_IDX = [1, 4, 7]


def _dtype(name: str) -> torch.dtype:
    # "fp8": the estimator's FC forward GEMM runs in OCP e4m3 (see HDCEModel); the convs and the
    # backward GEMMs compute in bf16
    return {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16, "fp8": torch.bfloat16}[name]


class HDCEModel:
    """3 scenario experts (Conv_P128) + shared FC_P128, stored grouped for one-kernel-per-layer
    execution.  The reference modules stay the single source of parameters (their tensors are
    views into the flat buffer), so ``Conv0.state_dict()`` etc. remain reference-compatible."""

    def __init__(self, pilot_num: int = 128, device="cpu", dtype: str = "bf16", n_experts: int = 3,
                 grad_extra: int = 0, fc_pad_multiple: int = 1, front: int = 0):
        """``fc_pad_multiple``: pad the flat space after the FC parameters so that the FC region
        [FC.weight offset, end) has a multiple of this many elements (ZeRO-1 sharding over ranks).
        ``front``: floats reserved in front of the flat space in the same allocation
        (``space.front_views``; FlatParamSpace)."""
        self.device = torch.device(device)
        self.E = n_experts
        self.H, self.W = pilot_grid(pilot_num)
        self.compute_dtype = _dtype(dtype) if self.device.type == "cuda" else torch.float32
        # fp8 estimator: FC forward = e4m3 x e4m3 (fp32 accumulate) with delayed per-tensor scales; slot
        # 0 = FC activations (quantised by the conv stack's last BN+ReLU kernel), slot 1 = FC weights
        # (quantised by the optimizer's shadow write), slots 2..5 = the e4m3 convs of layers 2 / 3
        # (activation, weight), slot 6 = the loss gradient dY (the e4m3 FC backward GEMMs) -- one scale-update
        # launch per step for all seven
        self.fp8 = dtype == "fp8" and self.device.type == "cuda"
        self.fp8_scales = None
        if self.fp8:
            from ..ops.optim import Fp8Scales
            self.fp8_scales = Fp8Scales(7, self.device)
        self.convs = [Conv_P128(pilot_num).to(self.device) for _ in range(n_experts)]
        self.fc = FC_P128(pilot_num).to(self.device)
        named = []
        for pname in CONV_PARAM_ORDER:
            for e, m in enumerate(self.convs):
                named.append((f"Conv{e}.{pname}", m.get_parameter(pname)))
        named += [("CE.FC.weight", self.fc.FC.weight), ("CE.FC.bias", self.fc.FC.bias)]
        if fc_pad_multiple > 1:
            al = lambda n: (n + ALIGN - 1) // ALIGN * ALIGN
            fc_len = al(self.fc.FC.weight.numel()) + al(self.fc.FC.bias.numel()) + al(grad_extra)
            grad_extra += (-fc_len) % (fc_pad_multiple * ALIGN)   # (every shard ALIGN-aligned)
        self.space = FlatParamSpace(named, self.device, extra=grad_extra, front=front)
        # grouped leaf views over the expert-consecutive parameter blocks
        self.conv_w, self.bn_w, self.bn_b = [], [], []
        for k in range(3):
            self.conv_w.append(self._group_leaf(f"Conv0.cnn.{3 * k}.weight"))
            self.bn_w.append(self._group_leaf(f"Conv0.cnn.{3 * k + 1}.weight"))
            self.bn_b.append(self._group_leaf(f"Conv0.cnn.{3 * k + 1}.bias"))
        self.fc_w = self._leaf(self.fc.FC.weight)
        self.fc_b = self._leaf(self.fc.FC.bias)
        # grouped BN running statistics; the modules' buffers become views
        C = 32 * n_experts
        self.run_mean = [torch.zeros(C, device=self.device) for _ in range(3)]
        self.run_var = [torch.ones(C, device=self.device) for _ in range(3)]
        for k, idx in enumerate(BN_IDX):
            for e, m in enumerate(self.convs):
                bn = m.cnn[idx]
                bn.running_mean = self.run_mean[k][e * 32:(e + 1) * 32]
                bn.running_var = self.run_var[k][e * 32:(e + 1) * 32]
        # all 3x3 num_batches_tracked counters are views of one int64 buffer: one add per step
        self._nbt = torch.zeros(n_experts * len(BN_IDX), dtype=torch.long, device=self.device)
        for e, m in enumerate(self.convs):
            for k, idx in enumerate(BN_IDX):
                m.cnn[idx].num_batches_tracked = self._nbt[e * len(BN_IDX) + k]
        self.nbt = [self._nbt]
        self.momentum, self.eps = 0.1, 1e-5
        self.fc_shadow: Optional[torch.Tensor] = None  # bf16 FC weight+bias kept fresh by the optimizer

    def attach_fc_shadow(self, opt, to_end: bool = False) -> None:
        """Let ``opt`` maintain a bf16 copy of the FC weight and bias (GPU, bf16 compute only);
        ``to_end``: the shadow spans the whole FC region up to the end of the flat space (sharded)."""
        if self.device.type != "cuda" or self.compute_dtype != torch.bfloat16:
            return
        lo = self.space.offsets[self.space.names.index("CE.FC.weight")]
        ob = self.space.offsets[self.space.names.index("CE.FC.bias")]
        hi = ob + self.fc_b.numel()
        hi = self.space.numel if to_end else hi + (-hi) % 4
        sh = opt.attach_shadow(lo, hi, fp8=self.fp8_scales, fp8_slot=1)
        self.fc_shadow = sh
        self._shadow_w = sh[:self.fc_w.numel()].view(self.fc_w.shape)
        self._shadow_b = sh[ob - lo:ob - lo + self.fc_b.numel()]
        if self.fp8:
            self._shadow_w8 = opt.shadow8[:self.fc_w.numel()].view(self.fc_w.shape)

    def fc_weights_lp(self):
        """(W, b) in the compute dtype: the optimizer-maintained shadow, or a fresh cast."""
        if self.fc_shadow is not None:
            return self._shadow_w, self._shadow_b
        dt = self.compute_dtype
        return self.fc_w.detach().to(dt), self.fc_b.detach().to(dt)

    # ------------------------------------------------------------------ params
    def _group_leaf(self, first_name: str) -> torch.Tensor:
        i = self.space.names.index(first_name)
        p0 = self.space.params[i]
        o = self.space.offsets[i]
        n = p0.numel() * self.E
        shape = (p0.shape[0] * self.E,) + tuple(p0.shape[1:])
        leaf = self.space.flat[o:o + n].view(shape)
        leaf.requires_grad_(True)
        leaf.grad = self.space.grad[o:o + n].view(shape)
        return leaf

    def _leaf(self, p: torch.Tensor) -> torch.Tensor:
        sl = self.space.slice_of(p)
        leaf = self.space.flat[sl].view(p.shape)
        leaf.requires_grad_(True)
        leaf.grad = self.space.grad[sl].view(p.shape)
        return leaf

    def modules(self) -> List[nn.Module]:
        return list(self.convs) + [self.fc]

    def train(self, mode: bool = True):
        for m in self.modules():
            m.train(mode)
        return self

    def eval(self):
        return self.train(False)

    def count_batches(self, n: int) -> None:
        with torch.no_grad():
            self._nbt.add_(n)

    # ------------------------------------------------------------------ forward pieces
    def pack_input(self, Yp: torch.Tensor) -> torch.Tensor:
        """(E, U, B, 2, H, W) stream-major pilots -> (U*B, E*2, H, W) grouped-conv input."""
        E, U, B = Yp.shape[:3]
        return Yp.permute(1, 2, 0, 3, 4, 5).reshape(U * B, E * 2, self.H, self.W)

    def conv_stack(self, x: torch.Tensor, n_groups: int, training: bool) -> torch.Tensor:
        """Grouped 3-layer conv/BN/ReLU; BN statistics per (sample group, channel)."""
        dt = self.compute_dtype
        h = x.to(dt)
        for k in range(3):
            z = F.conv2d(h, self.conv_w[k].to(dt), padding=1, groups=self.E)
            h = self._ghost_bn_relu(z, k, n_groups, training).to(dt)
        return h

    def _ghost_bn_relu(self, z: torch.Tensor, k: int, U: int, training: bool) -> torch.Tensor:
        NB, C, H, W = z.shape
        zf = z.float().view(U, NB // U, C, H * W)
        if training:
            var, mean = torch.var_mean(zf, dim=(1, 3), unbiased=False, keepdim=True)  # (U,1,C,1)
            with torch.no_grad():
                n = zf.shape[1] * zf.shape[3]
                unb = var.view(U, C) * (n / max(n - 1, 1))
                rm, rv = self.run_mean[k], self.run_var[k]
                for u in range(U):  # sequential updates = the reference's per-stream calls
                    rm.mul_(1 - self.momentum).add_(mean.view(U, C)[u], alpha=self.momentum)
                    rv.mul_(1 - self.momentum).add_(unb[u], alpha=self.momentum)
        else:
            mean = self.run_mean[k].view(1, 1, C, 1)
            var = self.run_var[k].view(1, 1, C, 1)
        y = (zf - mean) * torch.rsqrt(var + self.eps) * self.bn_w[k].view(1, 1, C, 1) + self.bn_b[k].view(1, 1, C, 1)
        return F.relu(y).view(NB, C, H, W)

    def fc_forward(self, a: torch.Tensor) -> torch.Tensor:
        dt = self.compute_dtype
        if self.fp8:   # evaluation in the training precision: on-the-fly per-tensor e4m3 scales
            return fp8_linear(a, self.fc_w.detach(), self.fc_b.detach().to(dt))
        return F.linear(a.to(dt), self.fc_w.to(dt), self.fc_b.to(dt))

    def features(self, Yp: torch.Tensor, training: bool) -> torch.Tensor:
        """(E, U, B, 2, H, W) -> FC operand (U*B*E, 32*H*W), rows ordered (u, b, e)."""
        E, U, B = Yp.shape[:3]
        h = self.conv_stack(self.pack_input(Yp), U, training)
        return h.reshape(U * B * E, 32 * self.H * self.W)

    @staticmethod
    def row_stream(E: int, U: int, B: int, device) -> torch.Tensor:
        """stream id (e*U + u) of every FC row in (u, b, e) order."""
        u = torch.arange(U, device=device).view(U, 1, 1)
        e = torch.arange(E, device=device).view(1, 1, E)
        return (e * U + u).expand(U, B, E).reshape(-1).to(torch.int32)

    @staticmethod
    def rows_from_streams(t: torch.Tensor) -> torch.Tensor:
        """(E, U, B, D) stream-major tensor -> (U*B*E, D) in FC row order."""
        E, U, B, D = t.shape
        return t.permute(1, 2, 0, 3).reshape(U * B * E, D)

    # ------------------------------------------------------------------ expert routing (eval)
    @torch.no_grad()
    def estimate_routed(self, x: torch.Tensor, expert: torch.Tensor) -> torch.Tensor:
        return estimate_routed(self.convs, self.fc, x, expert)


@torch.no_grad()
def estimate_routed(convs: Sequence[nn.Module], fc: nn.Module, x: torch.Tensor, expert: torch.Tensor,
                    chunk: int = 4096) -> torch.Tensor:
    """Test-time hierarchical routing (Test.py:166-214): sample i -> Conv_{expert[i]} -> shared CE.

    MoE-style top-1 routing: samples are bucketed by expert with ONE stable sort (the
    reference loops over samples in Python), each bucket runs through its expert, and the
    outputs are scattered back to input order."""
    E = len(convs)
    order = torch.argsort(expert, stable=True)
    counts = torch.bincount(expert, minlength=E).tolist()
    xs = x[order]
    out = torch.empty(x.shape[0], fc.FC.out_features, device=x.device, dtype=torch.float32)
    start = 0
    for e, c in enumerate(counts):
        for s in range(start, start + c, chunk):
            t = min(s + chunk, start + c)
            h = convs[e](xs[s:t].float())
            out[order[s:t]] = fc(h).float()
        start += c
    return out


class HDCEStep:
    """One fused HDCE training step over 9 stream batches (see module docstring).

    GPU path (``hip=True``): the conv/BN/ReLU stack runs on the hand-written kernels of
    csrc/hip/conv.hip with a manual backward, the FC on hipBLASLt (bf16 operands, fp32
    weight-gradient output written straight into the flat gradient buffer), the loss on
    csrc/hip/nmse.hip.  CPU / reference path: the same math through torch autograd."""

    def __init__(self, model: HDCEModel, n_users: int, batch: int, grad_hook: Optional[Callable] = None,
                 hip: Optional[bool] = None, skip: Optional[torch.Tensor] = None):
        """On the HIP path every gradient of the model is WRITTEN by exactly one kernel or GEMM
        (FC: GEMM out= / sum out=, conv + BN: overwrite mode) -- ``writes_grads`` -- so callers may
        skip zero_grad; the CPU/autograd path accumulates as usual."""
        self.m = model
        self.U, self.B = n_users, batch
        dev = model.device
        self.nmse = StreamNMSE(HDCEModel.row_stream(model.E, n_users, batch, dev), model.E * n_users)
        if skip is not None:  # share a NaN-guard flag (e.g. one that rides in a gradient bucket)
            self.nmse.skip = skip
        self.grad_hook = grad_hook  # called as grad_hook("fc") / grad_hook("conv") when buckets are final
        self.hip = (dev.type == "cuda") if hip is None else hip
        self.writes_grads = self.hip
        self.fused_nmse = True  # HIP path: the one-pass NMSE (qd_nmse_fused) when labels come via rowoff
        self.defer_dgrad = False
        # (world 1, GPU) FusedAdam: the FC weight's Adam step runs in the weight-gradient GEMM's epilogue
        # (ops/fc.gemm_wgrad_adam) -- dW is never written; the data gradient then runs first (it reads the
        # bf16 weight copy the fused update rewrites)
        self.fused_adam = None
        self.after_dgrad = None   # callable run right after the FC data gradient's launch (FlagshipConfig.fc_adam_side)
        # world-1 plans: the FC bias gradient's column reduction rides in the conv backward's slab launch
        # (never in DP: the FC gradient bucket is all-reduced before the conv backward runs)
        self.bias_via_conv_slabs = False
        # (world 1) backward_conv leaves the step's gradient slab reductions to the optimizer update (take_slabs)
        self.defer_slabs = False
        self._deferred = None
        self.defer_loss = True   # (with bias_via_conv_slabs) loss finish hosted by the conv backward
        self.stage_hook = None  # optional callable(stage) between forward launches (stream forks)
        # the FC GEMMs: hand-written MFMA kernels (csrc/hip/gemm.hip; knobs.KNOBS.hand_gemm = "": hipBLASLt) and
        # their tile configurations (forward, wgrad, dgrad; knobs.KNOBS.gemm_cfg).  Default: all three hand-written,
        # round 5: the producer-wave tiles (cfg 8, 7, 6) and the forward with the loss in its epilogue ("fwd", see
        # knobs.py); the round-4 notes below are the history of that choice --
        #   forward  "fwdplain", cfg 6: 192 x 128 tiles on a 4-stage LDS ring (round 4: two tiles in flight behind
        #            the MFMAs; isolated 43.5 vs 50.2 us for the 3-stage cfg 1, in the step 0.4012 / 0.3999 vs
        #            0.4070 / 0.4068 ms, profiles/r4_16_*); 192 workgroups, so ~64 CUs stay free for the concurrent
        #            QSC branch (hipBLASLt's 234-tile MT128x160 kernel leaves 22); bias-only epilogue, the loss as
        #            the separate one-pass NMSE kernel: 0.4095 / 0.4093 vs 0.4092 / 0.4070 ms with hipBLASLt (same
        #            box, profiles/r3_17_fwd192.txt); with 256 tiles (cfg 0 / 2) 0.8-1.3 % slower (r3_16), with the
        #            loss in the GEMM's epilogue ("fwd") 1.5-4 % slower (r3_02, r3_17): it keeps whole CUs from the
        #            QSC backward that then lands on the weight gradient;
        #   wgrad    cfg 1: 128 x 256 tiles, 8 waves (the 4-stage 128 x 128 cfg 4: 0.4103 / 0.4109 ms, slower);
        #   dgrad    cfg 2: 144 x 256 tiles, 8 waves along N (0.4115 /
        #            0.4116 vs 0.4180 / 0.4161 ms with the hipBLASLt data gradient, r3_02_gemm_variants.txt)
        hg = KNOBS.hand_gemm.strip()
        hg = {"1": "fwd,wgrad,dgrad", "all": "fwd,wgrad,dgrad", "0": "", "none": ""}.get(hg, hg)
        self.hand_gemm = set(x for x in hg.split(",") if x) if self.hip else set()
        assert self.hand_gemm <= {"fwd", "fwdplain", "wgrad", "dgrad"}, self.hand_gemm
        self.gemm_cfg = tuple(int(c) for c in KNOBS.gemm_cfg.split(","))
        # fp8 estimator: the FC weight / data gradients in e4m3 as well (see _fc_hand_f8; KNOBS.f8_bwd)
        self.f8_bwd = KNOBS.f8_bwd
        self.dgrad_bnred = False
        if self.hip:
            from ..ops.conv import ConvStackHIP
            self.conv = ConvStackHIP(model, n_users, batch, spw=KNOBS.conv_spw,
                                     spb_f=KNOBS.conv_spb_f_w16 if model.W == 16 else KNOBS.conv_spb_f,
                                     spb_w1=KNOBS.conv_spb_w1)
            self.conv.count_batches = True   # num_batches_tracked advanced inside the first BN launch
            self.fc_b_lp = None
            # layer 3's BN backward reduction in the FC data gradient's epilogue (ops.fc.gemm_dgrad_bnred): one
            # launch fewer on the chain (the bf16 hand-written dgrad, 3 experts, 144-row tiles within 2 groups)
            self.dgrad_bnred = bool(KNOBS.dgrad_bnred and "dgrad" in self.hand_gemm and not getattr(model, "fp8", False)
                                    and self.conv.bwd_fused and self.gemm_cfg[2] in (0, 2, 5, 6) and model.E == 3
                                    and self.conv.HW in (128, 256) and 3 * batch >= 144
                                    and (n_users * batch * 3) % 144 == 0)
            # the fp8 estimator's e4m3 data gradient with the same epilogue (gemm.hip qd_gemm_dgrad_f8_bnred,
            # 128-pixel maps only; KNOBS.dgrad_bnred_f8)
            if (KNOBS.dgrad_bnred_f8 and getattr(model, "fp8", False) and KNOBS.hand_fp8 and self.conv.bwd_fused
                    and model.E == 3 and self.conv.HW == 128 and 3 * batch >= 144
                    and (n_users * batch * 3) % 144 == 0):
                M = n_users * batch * 3
                self.dgrad_bnred = self._f8_bwd_ok(M, model.fc_w.shape[0], model.fc_w.shape[1])
            if self.dgrad_bnred:
                self.conv.enable_dgrad_bnred(n_users * batch * 3 // 144)

    def prime_fp8_dy(self, forward: Callable[[], Optional["HDCEStep"]], state: Sequence[torch.Tensor], ctx=None,
                     engines: Sequence["HDCEStep"] = ()) -> bool:
        """(fp8 estimator with e4m3 FC gradients) seed the delayed scale of the loss gradient dY (fp8 slot 6).
        The loss epilogue quantises dY with the PREVIOUS step's scale, and dY = 2 err / (S den) sits far below
        e4m3's range at the initial unit scale: the first step's FC gradients would underflow.
        ``forward`` runs one forward + loss pass (this step's bf16-gradient path) on the first batch and returns
        the engine that ran it -- with several part sizes (runner.py) a rank's part may use another engine than
        this one -- or None when this rank's part is empty (it then contributes amax 0).  ``engines``: every
        engine forward may dispatch to (all are switched to bf16 gradients for the pass).  max |dY| (max over
        ranks with ``ctx``: every rank enters the collective) sets the slot; every tensor in ``state`` is
        restored afterwards, so the run differs from an unprimed one only in slot 6.  Returns whether it primed."""
        sc = getattr(self.m, "fp8_scales", None)
        if sc is None or not self.hip or not self.f8_bwd:
            return False
        engs = list(dict.fromkeys([self, *engines]))
        saved = [t.clone() for t in state]
        flags = [e.f8_bwd for e in engs]
        for e in engs:
            e.f8_bwd = False
        try:
            used = forward()
            if used is None:
                amax = torch.zeros(1, device=sc.amax.device, dtype=torch.float32)
            else:
                amax = used._dYW[0].detach().abs().amax().float().view(1)
            if ctx is not None and ctx.distributed:
                ctx.all_reduce_(amax, "max")
            amax = amax.clamp_min(1e-30)
        finally:
            for e, f in zip(engs, flags):
                e.f8_bwd = f
            for t, c in zip(state, saved):
                t.copy_(c)
        sc.set_from_tensor(6, amax)
        return True

    def __call__(self, Yp: torch.Tensor, HL: torch.Tensor, HP: torch.Tensor) -> torch.Tensor:
        """Yp (E,U,B,2,H,W), HL/HP (E,U,B,2048) fp32.  Returns device loss[2] (loss, loss_perf)."""
        loss = self.forward_fc(Yp, HL, HP)
        if self.grad_hook:
            self.grad_hook("fc")
        self.backward_conv()
        if self.grad_hook:
            self.grad_hook("conv")
        return loss

    # Phase 1: forward, fused NMSE, complete FC backward (FC grads final, dA ready).
    def forward_fc(self, Yp: torch.Tensor, HL: torch.Tensor, HP: torch.Tensor) -> torch.Tensor:
        """From stream-major tensors Yp (E,U,B,2,H,W), HL/HP (E,U,B,2048)."""
        self.nmse.rowoff = None
        x1 = self.m.pack_input(Yp).float().contiguous()
        return self._forward_fc(x1, HDCEModel.rows_from_streams(HL), HDCEModel.rows_from_streams(HP))

    def forward_fc_gathered(self, g, store) -> torch.Tensor:
        """From a filled ops.gather.StepGather: conv input g.x1, labels read in place from the
        store through g.rowoff (no permuted label copies)."""
        self.nmse.rowoff = g.rowoff
        self._rowden = g.rowden if getattr(g, "rowpow", None) is not None else None
        self._apply_den_global()
        return self._forward_fc(g.x1, store.Hlabel, store.Hperf)

    def _apply_den_global(self) -> None:
        """(DataParallel semantics) this rank holds part of each stream's batch: scale its per-row label
        powers so that the one-pass NMSE kernels' per-stream sums ARE the global batch's denominators."""
        dg = self.nmse.den_global
        if dg is None or self._rowden is None:
            return
        rs = self.nmse._rs_long
        loc = torch.zeros(self.nmse.S, 2, device=dg.device).index_add_(0, rs, self._rowden)
        self._rowden.mul_((dg / loc.clamp_min(1e-30))[rs])

    # the same forward in two halves (HIP path; the DP plan replays them as separate graphs, so the FC
    # weights' update from the previous step -- an all-gather or the FC Adam -- overlaps the conv forward)
    def forward_conv_gathered(self, g) -> None:
        """Half 1: the conv / BN / ReLU stack on g.x1 (no FC weight read)."""
        assert self.hip
        self.nmse.rowoff = g.rowoff
        self._rowden = g.rowden if getattr(g, "rowpow", None) is not None else None
        self._apply_den_global()
        self.conv.stage_hook = self.stage_hook
        self._A_conv = self.conv.forward(g.x1, training=True)
        if self.stage_hook is not None:
            self.stage_hook("conv")

    def forward_fc_after_conv(self, store) -> torch.Tensor:
        """Half 2: FC forward, loss, FC weight gradient (+ data gradient unless deferred)."""
        # (the conv output is a static buffer: graph capture replays this half on its own several times)
        return self._fc_hip(self._A_conv, store.Hlabel, store.Hperf)

    def _forward_fc(self, x1: torch.Tensor, label: torch.Tensor, perf: torch.Tensor) -> torch.Tensor:
        if self.hip:
            return self._forward_fc_hip(x1, label, perf)
        m = self.m
        A = m.conv_stack(x1, self.U, training=True).reshape(x1.shape[0] * m.E, -1)
        A_det = A.detach().requires_grad_(True)
        Y = m.fc_forward(A_det)
        loss = self.nmse.sums_finalize(Y, label, perf)
        dY = self.nmse.grad(Y, label, out_dtype=Y.dtype)
        torch.autograd.backward(Y, dY)             # FC grads + dA
        self._A, self._dA = A, A_det.grad
        return loss

    # Phase 2: conv/BN backward from dA.
    def backward_conv(self, slabs=None, side=None) -> None:
        """``slabs``: queue the conv weight-gradient reductions on this ``SlabBatch`` (HIP path; the
        caller launches it in overwrite mode).  ``side``: stream for the conv weight-gradient kernels
        (see ConvStackHIP.backward)."""
        if self.hip:
            pending = getattr(self, "_slabs", None)
            self._slabs = None
            lf = getattr(self.nmse, "pending_finish", None)
            self.nmse.pending_finish = None
            if pending is not None and slabs is None:
                # the conv weight / BN slabs and the pending FC bias reduction: one overwrite launch -- or (defer_slabs)
                # none: the caller's optimizer update sums them itself (take_slabs)
                self.conv.backward(self._dA, accumulate=False, slabs=pending, side=side, loss_finish=lf)
                if self.defer_slabs:
                    self._deferred = pending
                else:
                    pending.launch(accumulate=False, stream=nat.stream_ptr(self._dA.device))
            else:
                if pending is not None:
                    pending.launch(accumulate=False, stream=nat.stream_ptr(self._dA.device))
                self.conv.backward(self._dA, accumulate=False, slabs=slabs, side=side, loss_finish=lf)
        else:
            torch.autograd.backward(self._A, self._dA)
            self._A = None
        if not (self.hip and self.conv.count_batches):   # the HIP forward counted them in-kernel
            self.m.count_batches(self.U)

    def take_slabs(self):
        """(defer_slabs) the SlabBatch the last backward_conv left unlaunched -- the conv weight / BN gradient slabs and
        the FC bias reduction -- for ``FusedOptimizer.step(slabs=...)``; None when there is none."""
        b, self._deferred = self._deferred, None
        return b

    @torch.no_grad()
    def _forward_fc_hip(self, x1: torch.Tensor, label: torch.Tensor, perf: torch.Tensor) -> torch.Tensor:
        hook = self.stage_hook
        self.conv.stage_hook = hook
        A = self.conv.forward(x1, training=True)                # (rows, 4096) bf16
        if hook is not None:
            hook("conv")
        return self._fc_hip(A, label, perf)

    def _hand_gemm_ok(self, A: torch.Tensor) -> bool:
        """The hand-written FC GEMMs (csrc/hip/gemm.hip) apply: bf16 estimator, labels gathered through
        rowoff with per-row powers, a shape the kernels tile (knobs.KNOBS.hand_gemm without "fwd": hipBLASLt)."""
        m = self.m
        if not ("fwd" in self.hand_gemm and m.compute_dtype == torch.bfloat16 and not m.fp8 and self.nmse.rowoff is not None
                and getattr(self, "_rowden", None) is not None):
            return False
        from ..ops.fc import gemm_fwd_ok, gemm_tile_m
        M, K = A.shape
        N = m.fc_w.shape[0]
        c = self.gemm_cfg
        tm = gemm_tile_m(c[0])
        return (gemm_fwd_ok(M, N, K, c[0]) and N % 256 == 0 and M % 128 == 0 and K % 256 == 0
                and (tm // (self.B * m.E) + 2) * m.E <= 64 and self.B % 16 == 0 and tm % (16 * m.E) == 0)

    @torch.no_grad()
    def _fc_hand(self, A: torch.Tensor, label: torch.Tensor, perf: torch.Tensor) -> torch.Tensor:
        """FC forward with the loss fused into its epilogue, then the weight and data gradients -- all
        three GEMMs hand-written (csrc/hip/gemm.hip), no Y in memory."""
        from ..ops.fc import gemm_dgrad, gemm_wgrad
        from ..ops.slabsum import SlabBatch
        m = self.m
        W, b = m.fc_weights_lp()
        self._slabs = SlabBatch() if (self.writes_grads and self.bias_via_conv_slabs) else None
        dY = self.nmse.gemm_fused(A, W, b, label, perf, m.fc_b.grad, (m.E, self.U, self.B), self._rowden,
                                  bias_slabs=self._slabs, defer_loss=self._slabs is not None and self.defer_loss,
                                  cfg=self.gemm_cfg[0])
        if self.stage_hook is not None:
            self.stage_hook("fc")
        self._fc_backward(dY, A, W)
        return self.nmse.loss

    def _fc_backward(self, dY: torch.Tensor, A: torch.Tensor, W: torch.Tensor) -> None:
        """The FC weight gradient (or its fused Adam step) and the data gradient (unless deferred)."""
        self._dYW = (dY, W)
        if self.fused_adam is not None:
            assert not self.defer_dgrad
            self.dgrad()
            self._wgrad(dY, A)
            return
        self._wgrad(dY, A)
        if not self.defer_dgrad:
            self.dgrad()

    def _plain_fwd_ok(self, A: torch.Tensor, W: torch.Tensor) -> bool:
        from ..ops.fc import gemm_fwd_ok
        return A.is_contiguous() and W.is_contiguous() and gemm_fwd_ok(A.shape[0], W.shape[0], A.shape[1],
                                                                        self.gemm_cfg[0])

    def _hand_f8_ok(self, A: torch.Tensor) -> bool:
        """The fp8 estimator's forward on the hand-written e4m3 GEMM with the loss epilogue
        (qd_gemm_fwd_nmse_f8): e4m3 activations from the conv stack, e4m3 weight shadow from the
        optimizer, rowoff-gathered labels.  KNOBS.hand_fp8 False: hipBLASLt (torch._scaled_mm) + the NMSE kernel."""
        m = self.m
        if not (m.fp8 and m.fc_shadow is not None and KNOBS.hand_fp8
                and self.nmse.rowoff is not None and getattr(self, "_rowden", None) is not None
                and getattr(self.conv, "h3_8", None) is not None):
            return False
        from ..ops.fc import gemm_tile_m
        M, K = A.shape
        N = m.fc_w.shape[0]
        tm = gemm_tile_m(0)
        return (M % tm == 0 and N % 128 == 0 and K % 128 == 0 and (tm // (self.B * m.E) + 2) * m.E <= 64
                and self.B % 16 == 0 and tm % (16 * m.E) == 0)

    def _f8_bwd_ok(self, M: int, N: int, K: int) -> bool:
        """The FC weight / data gradients in e4m3 too (KNOBS.f8_bwd False: bf16): shapes the MX-scaled GEMMs tile
        (dgrad 144 x 128 tiles over K = N, wgrad 128 x 256 tiles over K = M)."""
        return self.f8_bwd and M % 256 == 0 and N % 256 == 0 and K % 256 == 0 and M % 144 == 0

    @torch.no_grad()
    def _fc_hand_f8(self, A: torch.Tensor, label: torch.Tensor, perf: torch.Tensor) -> torch.Tensor:
        """fp8 estimator: e4m3 forward GEMM with the loss fused into its epilogue (per-tensor delayed
        scales of the previous step).  The weight and data gradients run in e4m3 as well when the shapes allow
        (_f8_bwd_ok): the loss epilogue also writes dY as e4m3 (delayed scale slot 6), and both gradients run on
        the MX-scaled MFMA straight from the row-major e4m3 tensors -- dW = dY8^T A8 and dA = dY8 W8, the
        i-contiguous operands read through ds_read_b64_tr_b8, no transposed copies; else bf16 gradients.  The
        scale update runs after the data gradient then (every e4m3 operand of the step is dequantised with the
        scale it was quantised with)."""
        from ..ops.slabsum import SlabBatch
        m = self.m
        W, b = m.fc_weights_lp()
        M, K = A.shape
        N = m.fc_w.shape[0]
        bwd8 = self._f8_bwd_ok(M, N, K)
        f8o = None
        sc = m.fp8_scales
        if bwd8:
            if getattr(self, "_dY8", None) is None or self._dY8.shape != (M, N):
                self._dY8 = torch.empty(M, N, device=A.device, dtype=torch.float8_e4m3fn)
            f8o = (self._dY8, None, sc.qs[6:7], sc.amax[6])
        self._slabs = SlabBatch() if (self.writes_grads and self.bias_via_conv_slabs) else None
        dY = self.nmse.gemm_fused(self.conv.h3_8, m._shadow_w8, b, label, perf, m.fc_b.grad, (m.E, self.U, self.B),
                                  self._rowden, bias_slabs=self._slabs,
                                  defer_loss=self._slabs is not None and self.defer_loss, deq=sc.scale, f8_out=f8o)
        if not bwd8:
            sc.update()
        if self.stage_hook is not None:
            self.stage_hook("fc")
        self._f8_bwd = bwd8
        if bwd8:
            from ..ops.fc import gemm_wgrad_f8
            gemm_wgrad_f8(self._dY8, self.conv.h3_8.view(M, K), sc.scale[6:7], sc.scale[0:1], out=m.fc_w.grad,
                          cfg=int(KNOBS.f8_producers))
        else:
            self._wgrad(dY, A.to(m.compute_dtype))
        self._dYW = (dY, W)
        if not self.defer_dgrad:
            self.dgrad()
        return self.nmse.loss

    @torch.no_grad()
    def _fc_hip(self, A: torch.Tensor, label: torch.Tensor, perf: torch.Tensor) -> torch.Tensor:
        if self.stage_hook is not None:
            self.stage_hook("fc_pre")   # (before anything reads the FC weights)
        if self._hand_gemm_ok(A):
            self.fc_path = "hand"
            return self._fc_hand(A, label, perf)
        if self._hand_f8_ok(A):
            self.fc_path = "hand_f8"
            return self._fc_hand_f8(A, label, perf)
        self.fc_path = "library"   # (which FC forward the last step ran: hand / hand_f8 / library)
        m = self.m
        dt = m.compute_dtype
        hook = self.stage_hook
        W, b = m.fc_weights_lp()
        if m.fp8 and m.fc_shadow is None:
            Y = fp8_linear(A, m.fc_w.detach(), b)
        elif m.fp8:
            # fp8 forward GEMM: activations quantised by the conv stack's last kernel, weights by the
            # optimizer (both with the scales of the previous step); then the scales move on
            sc = m.fp8_scales.scale
            Y = torch._scaled_mm(self.conv.h3_8, m._shadow_w8.t(), scale_a=sc[0], scale_b=sc[1], bias=b,
                                 out_dtype=dt)
            m.fp8_scales.update()
        elif ("fwdplain" in self.hand_gemm or "fwd" in self.hand_gemm) and dt == torch.bfloat16 and A.dtype == dt \
                and W.dtype == dt and b is not None and b.dtype == dt and self._plain_fwd_ok(A, W):
            # the hand-written forward GEMM with only the bias in its epilogue; the loss runs as the separate
            # one-pass NMSE kernel below, as after a library GEMM.  ("fwd" too, for shapes the loss epilogue does not
            # tile, e.g. M % 128 != 0 at small batches: its hipBLASLt fallback broke the split-forward plans'
            # equality with the serial step -- profiles/r5_41_map.txt)
            from ..ops.fc import gemm_fwd
            if getattr(self, "_Y_buf", None) is None or self._Y_buf.shape != (A.shape[0], W.shape[0]):
                self._Y_buf = torch.empty(A.shape[0], W.shape[0], device=A.device, dtype=dt)
            Y = gemm_fwd(A, W, b, out=self._Y_buf, cfg=self.gemm_cfg[0])
            self.fc_path = "hand_plain"
        else:
            Y = torch.nn.functional.linear(A.to(dt), W, b)
        if hook is not None:
            hook("fc")
        if self.nmse.rowoff is not None and self.fused_nmse and self.nmse.cols % 1024 == 0:
            # one pass: loss, skip, dY, bias-gradient partials (+ one finish launch)
            # (the FC bias gradient's column reduction joins the conv backward's slab batch: one launch less
            # between the loss and the FC gradient GEMMs)
            from ..ops.slabsum import SlabBatch
            self._slabs = SlabBatch() if (self.writes_grads and self.bias_via_conv_slabs) else None
            # (with the bias in the conv slab batch, the loss finish rides in the conv backward too:
            # nothing between here and there reads loss or skip)
            dY = self.nmse.fused(Y, label, perf, m.fc_b.grad, (m.E, self.U, self.B), out_dtype=dt,
                                 rowden=getattr(self, "_rowden", None), bias_slabs=self._slabs,
                                 defer_loss=self._slabs is not None and self.defer_loss)
            loss = self.nmse.loss
        else:
            loss = self.nmse.sums_finalize(Y, label, perf)
            dY = self.nmse.grad_bias(Y, label, m.fc_b.grad, out_dtype=dt)   # + bias grad, same pass
        A = A.to(dt)
        self._fc_backward(dY, A, W)
        return loss

    def _wgrad(self, dY: torch.Tensor, A: torch.Tensor) -> None:
        """dW = dY^T A (fp32, straight into the flat gradient): the hand-written GEMM for bf16 operands of a
        tiled shape, else hipBLASLt."""
        from ..ops.fc import gemm_wgrad
        m = self.m
        from ..ops.fc import gemm_wgrad_ok
        hand = ("wgrad" in self.hand_gemm and dY.dtype == A.dtype == torch.bfloat16
                and gemm_wgrad_ok(dY.shape[0], dY.shape[1], A.shape[1], self.gemm_cfg[1]))

        fa = self.fused_adam
        if fa is not None and not hand:
            raise RuntimeError("the fused FC Adam needs the hand-written weight-gradient GEMM for this shape")

        def run():
            if fa is not None:
                from ..ops.fc import gemm_wgrad_adam
                gemm_wgrad_adam(dY, A, fa["opt"], fa["lo"], fa["slot"], skip=fa["skip"], cfg=self.gemm_cfg[1])
            elif hand:
                gemm_wgrad(dY, A, out=m.fc_w.grad, cfg=self.gemm_cfg[1])
            else:
                _mm_f32(dY.t(), A, m.fc_w.grad)

        run()

    def dgrad(self) -> None:
        """dA = dY W (HIP path): issued by the forward unless ``defer_dgrad`` (the DP plan issues it
        after the FC gradient all-reduce is on its way)."""
        dY, W = self._dYW
        from ..ops.fc import gemm_dgrad
        if getattr(self, "_f8_bwd", False):   # (fp8 estimator, see _fc_hand_f8)
            from ..ops.fc import gemm_dgrad_f8
            m = self.m
            sc = m.fp8_scales
            if getattr(self, "_dA_buf", None) is None or self._dA_buf.shape != (dY.shape[0], W.shape[1]):
                self._dA_buf = torch.empty(dY.shape[0], W.shape[1], device=dY.device, dtype=torch.bfloat16)
            if self.dgrad_bnred:
                from ..ops.fc import gemm_dgrad_f8_bnred
                c = self.conv
                self._dA = gemm_dgrad_f8_bnred(self._dY8, m._shadow_w8, sc.scale[6:7], sc.scale[1:2], self._dA_buf,
                                               int(KNOBS.f8_producers), c.z[2], c.st[2], c.rslab[2], self.B, self.U,
                                               c.HW)
            else:
                self._dA = gemm_dgrad_f8(self._dY8, m._shadow_w8, sc.scale[6:7], sc.scale[1:2], out=self._dA_buf,
                                         cfg=int(KNOBS.f8_producers))
            sc.update()
            if self.stage_hook is not None:
                self.stage_hook("dgrad")
            return
        from ..ops.fc import gemm_dgrad_ok
        if "dgrad" in self.hand_gemm and dY.dtype == torch.bfloat16 and W.dtype == torch.bfloat16 \
                and gemm_dgrad_ok(dY.shape[0], W.shape[0], W.shape[1], self.gemm_cfg[2]):
            if getattr(self, "_dA_buf", None) is None or self._dA_buf.shape != (dY.shape[0], W.shape[1]):
                self._dA_buf = torch.empty(dY.shape[0], W.shape[1], device=dY.device, dtype=torch.bfloat16)
            if self.dgrad_bnred:
                from ..ops.fc import gemm_dgrad_bnred
                c = self.conv
                self._dA = gemm_dgrad_bnred(dY, W, self._dA_buf, self.gemm_cfg[2], c.z[2], c.st[2], c.rslab[2],
                                            self.B, self.U, c.HW)
            else:
                self._dA = gemm_dgrad(dY, W, out=self._dA_buf, cfg=self.gemm_cfg[2])
        else:
            if self.dgrad_bnred:
                raise RuntimeError("dgrad_bnred needs the hand-written bf16 or e4m3 data gradient")
            self._dA = torch.mm(dY, W)                         # (rows, 4096) bf16
        if self.after_dgrad is not None:   # (the FC weight's shadow has had its last reader of the step)
            self.after_dgrad()
        if self.stage_hook is not None:
            self.stage_hook("dgrad")

    @property
    def skip(self) -> torch.Tensor:
        return self.nmse.skip


def fp8_linear(a: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ w.T + b with both operands quantised to OCP e4m3 (per-tensor scales computed here)."""
    from ..ops.optim import FP8_E4M3_MAX
    sa = (a.detach().abs().amax().float().clamp_min(1e-30) * 2.0 / FP8_E4M3_MAX).reshape(())
    sw = (w.abs().amax().float().clamp_min(1e-30) * 2.0 / FP8_E4M3_MAX).reshape(())
    a8 = (a.float() / sa).to(torch.float8_e4m3fn)
    w8 = (w.float() / sw).to(torch.float8_e4m3fn)
    return torch._scaled_mm(a8, w8.t(), scale_a=sa, scale_b=sw, bias=b, out_dtype=b.dtype)


def _mm_f32(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> None:
    """out = a @ b with low-precision operands and an fp32 result (hipBLASLt)."""
    if a.dtype == torch.float32:
        torch.mm(a, b, out=out)
    else:
        torch.mm(a, b, out_dtype=torch.float32, out=out)


class ClassifierStep:
    """One fused step of a scenario classifier (QSC_P128 or SC_P128) over all 9 streams.

    The reference sums 9 per-stream ``nll_loss / 9`` (R:362); with equal stream batches that
    is exactly the mean NLL over the concatenated 9*B samples, computed in one pass.
    For QSC with QuantumNAT on, each stream gets its own noise draw (the reference draws
    per forward call) through grouped quantum weights."""

    def __init__(self, model: nn.Module, n_streams: int, grad_hook: Optional[Callable] = None,
                 space: Optional[FlatParamSpace] = None, batch_total: Optional[int] = None,
                 skip: Optional[torch.Tensor] = None, hip_kw: Optional[dict] = None):
        """``skip``: a shared NaN-guard flag another loss already set this step (it is incremented);
        by default the step owns its flag (``self.skip``, overwritten every step).  ``hip_kw``: extra
        QSCStepHIP arguments (launch grids)."""
        self.model = model
        self.S = n_streams
        self.grad_hook = grad_hook
        dev0 = next(model.parameters()).device
        self.skip_add = skip is not None
        self.skip = skip if skip is not None else torch.zeros(1, device=dev0, dtype=torch.float32)
        self.writes_grads = False   # set by callers that skip zero_grad (fused HIP step only)
        self.hip = None
        dev = next(model.parameters()).device
        if (isinstance(model, QSC_P128) and model.use_quantum and dev.type == "cuda" and space is not None
                and batch_total):
            from ..ops.qsc import QSCStepHIP
            self.hip = QSCStepHIP(model, space, batch_total, n_groups=n_streams, **(hip_kw or {}))
        elif isinstance(model, SC_P128) and dev.type == "cuda" and space is not None:
            from ..ops.sc import SCStepHIP   # (any batch size: the kernels take B per call)
            self.hip = SCStepHIP(model, space, batch_total or 0)
        self.is_sc = isinstance(model, SC_P128)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """Inference log-probabilities.  GPU: the HIP kernels (the SC's fused forward; for the QSC the
        preprocess CNN + the circuit on the clean master weights + the inference head,
        QSCStepHIP.infer) in chunks of the step's static batch; else the models' torch forward."""
        m = self.model
        if self.is_sc and self.hip is not None:
            return self.hip.forward(x)
        if self.hip is not None and getattr(self.hip, "impl", None) == "mfma" and not m.training:
            return self._infer_hip(x)
        if isinstance(m, QSC_P128) and m.use_quantum:
            angles = m.preprocess(x)
            w = m.qlayer.weights
            if m.training and m.use_quantumnat and m.noise_level > 0:
                noise = torch.randn((self.S,) + tuple(w.shape), device=w.device, dtype=w.dtype)
                w = w.unsqueeze(0) + m.noise_level * noise
            xq = m.qlayer(angles, w)
            return F.log_softmax(m.classifier(xq), dim=1)
        return m(x)

    @torch.no_grad()
    def _infer_hip(self, x: torch.Tensor) -> torch.Tensor:
        """(QSC, GPU) log-probabilities of any number of samples through QSCStepHIP.infer, which runs exactly
        its static batch: chunks of that size, the last one padded by repeating its final sample."""
        h = self.hip
        Bs = h.B
        x = x.contiguous().float()
        N = x.shape[0]
        if getattr(self, "_xin", None) is None:
            self._xin = torch.empty((Bs,) + tuple(x.shape[1:]), device=x.device)
            self._logp = torch.empty(Bs, h.C, device=x.device)
        out = torch.empty(N, h.C, device=x.device)
        for lo in range(0, N, Bs):
            n = min(Bs, N - lo)
            self._xin[:n].copy_(x[lo:lo + n])
            if n < Bs:
                self._xin[n:].copy_(x[lo + n - 1:lo + n].expand(Bs - n, *x.shape[1:]))
            h.infer(self._xin, None, self._logp)
            out[lo:lo + n].copy_(self._logp[:n])
        return out

    def forward_part(self, x: torch.Tensor, labels: torch.Tensor) -> None:
        """(HIP path) the step's forward half: loss, NaN flag, head grads (see QSCStepHIP.forward_part)."""
        self.hip.forward_part(x.contiguous(), labels, skip=self.skip, skip_add=self.skip_add,
                              accumulate=not self.writes_grads)

    def backward_part(self, x: torch.Tensor, slabs=None) -> torch.Tensor:
        """(HIP path) the step's backward half; returns the loss."""
        loss = self.hip.backward_part(x.contiguous(), accumulate=not self.writes_grads, slabs=slabs)
        if self.grad_hook:
            self.grad_hook("all")
        return loss

    def __call__(self, x: torch.Tensor, labels: torch.Tensor, slabs=None) -> torch.Tensor:
        """``slabs`` (HIP path): queue the gradient-slab reductions on this ``SlabBatch`` (launched by
        the caller, with accumulate = not writes_grads)."""
        if self.hip is not None and (self.is_sc or x.shape[0] == self.hip.B):
            loss = self.hip(x.contiguous(), labels, skip=self.skip, skip_add=self.skip_add,
                            accumulate=not self.writes_grads, slabs=slabs)
            if self.grad_hook:
                self.grad_hook("all")
            return loss
        out = self.forward(x)
        loss = F.nll_loss(out, labels)
        loss.backward()
        bad = (~torch.isfinite(loss.detach())).float().reshape(1)
        if self.skip_add:
            self.skip.add_(bad)
        else:
            self.skip.copy_(bad)
        if self.grad_hook:
            self.grad_hook("all")
        return loss.detach()
