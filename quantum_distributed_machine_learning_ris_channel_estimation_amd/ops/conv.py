"""HIP conv-BN-ReLU stack of the HDCE experts (csrc/hip/conv.hip), forward + manual backward.

Reference module: ``Conv_P128.cnn`` (Estimators_QuantumNAT_onchipQNN.py:246-261) = 3 x
[Conv2d 3x3 no-bias -> BatchNorm2d(32) -> ReLU], one instance per scenario expert.

``ConvStackHIP`` runs all experts for a whole 9-stream step with 3 forward conv launches
(+3 tiny statistics launches, +1 weight-pack launch) and 3 x (BN reduce, BN finalize, dgrad, wgrad, slab sum)
backward launches; every buffer is allocated once, so the whole step is capturable in a
HIP graph.  Gradients are written straight into the model's flat gradient buffer.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from .. import _native as nat
from ..knobs import KNOBS
from .slabsum import SlabBatch

_p, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
NST = 8


def _ptr(t: Optional[torch.Tensor]):
    return nat.ptr(t) if t is not None else None


class BnFwd(ctypes.Structure):
    """csrc/hip/conv.hip ``BnFwd``: forward BN finalisation fused into the consuming conv kernel."""
    _fields_ = [("stats", _p), ("gamma", _p), ("beta", _p), ("run_mean", _p), ("run_var", _p), ("st_out", _p),
                ("chunks", _i), ("count", _f), ("momentum", _f), ("eps", _f), ("training", _i)]


class BnRed(ctypes.Structure):
    """csrc/hip/conv.hip ``BnRed``: the previous layer's BN backward reduction fused into dgrad."""
    _fields_ = [("z", _p), ("st", _p), ("part", _p)]


class StackFwd(ctypes.Structure):
    """csrc/hip/conv.hip ``StackFwd``: the persistent training forward's operands (conv_fwd_stack_kernel)."""
    _fields_ = [("x1", _p), ("w", _p * 3), ("z", _p * 3), ("stats", _p * 3), ("gamma", _p * 3), ("beta", _p * 3),
                ("run_mean", _p * 3), ("run_var", _p * 3), ("st", _p * 3), ("h3", _p), ("nbt", _p),
                ("nbt_inc", ctypes.c_longlong), ("count", _f), ("momentum", _f), ("eps", _f)]


class BnBwd(ctypes.Structure):
    """csrc/hip/conv.hip ``BnBwd``: BN backward finalisation fused into the wgrad / dgrad kernels."""
    _fields_ = [("rslab", _p), ("gamma", _p), ("chunks", _i), ("count", _f)]


class ConvStackHIP:
    """Grouped (experts-in-channels) 3-layer conv/BN/ReLU on (N, E*2, H, W) pilots."""

    def __init__(self, model, U: int, B: int, spw: int = 3, spb_w: int = 8, spb_r: int = 4, spb_w1: int = 4,
                 dx_bf16: bool = True, bwd_fused: Optional[bool] = None, spb_f: int = 5,
                 spb_db: Optional[int] = None):
        self.m = model
        self.count_batches = False   # set by the owner that stops counting num_batches_tracked itself
        self.stage_hook = None       # optional callable(stage name) between forward launches
        if not 1 <= U <= 8:
            raise ValueError(f"ConvStackHIP: {U} BatchNorm groups per step (1..8 supported)")
        self.U, self.B, self.N, self.E = U, B, U * B, model.E
        self.H, self.W = model.H, model.W
        self.HW = self.H * self.W
        self.EC = 32 * self.E
        dev = model.device
        self.spw = spw
        self.chunks = (B + 4 * spw - 1) // (4 * spw)          # forward / dgrad: 4 waves x spw samples
        self.spb_w = spb_w
        self.chunks_w = (B + spb_w - 1) // spb_w              # wgrad workgroups per group
        # backward of layers 3 and 2 (dx bf16): conv3x3_bwd_kernel computes wgrad, dgrad and the previous
        # layer's BN partials from ONE staging of each sample, spb_f samples per workgroup (5: 468
        # workgroups, two resident per CU, one staging while the other computes; 8 = 288 workgroups
        # left half the CUs with one and measured slower than the side-by-side wd kernel).
        # bwd_fused=False: wgrad and dgrad as separate workgroups of the wd kernel (tests compare the two).
        self.bwd_fused = (True if bwd_fused is None else bool(bwd_fused)) and dx_bf16
        # (round 6) P128: the fused backward software-pipelined over two stage buffers (conv3x3_bwd_db_kernel), one
        # workgroup per CU with spb_db samples each (bit-identical to conv3x3_bwd_kernel at the same chunking)
        self.bwd_db = self.bwd_fused and bool(KNOBS.conv_bwd_db) and model.H == 16 and model.W == 8
        if self.bwd_db:
            spb_f = KNOBS.conv_spb_db if spb_db is None else spb_db
        # layer 1 (2 input channels) is one accumulator tile: staging-bound, so more, shorter workgroups
        self.spb_wl = (spb_w1, spb_f, spb_f) if self.bwd_fused else (spb_w1, spb_w, spb_w)
        self.chunks_wl = tuple((B + s - 1) // s for s in self.spb_wl)
        self.spb_r = spb_r
        self.chunks_r = (B + spb_r - 1) // spb_r              # BN backward reductions
        N, EC, HW = self.N, self.EC, self.HW
        bf = torch.bfloat16
        self.z = [torch.empty(N, EC, HW, device=dev, dtype=bf) for _ in range(3)]
        self.h3 = torch.empty(N * self.E, 32 * HW, device=dev, dtype=bf)
        self.fp8 = getattr(model, "fp8", False)
        self.h3_8 = torch.empty(N * self.E, 32 * HW, device=dev, dtype=torch.float8_e4m3fn) if self.fp8 else None
        # fp8 estimator: the 32-channel forward convs (layers 2, 3) on e4m3 MFMA (conv3x3_f8_kernel) with
        # delayed per-tensor scales: slots 2..5 = [act2, w2, act3, w3] of the model's Fp8Scales (updated
        # with the FC's).  Opt-in (knobs.KNOBS.fp8_conv): in the step the e4m3 convs are no faster than the bf16 ones
        # (latency-bound 32-channel layers; the weight quantisation sits in their prologue), so the default fp8
        # estimator runs the FC -- 78 % of the HDCE FLOPs -- in e4m3 (forward, weight and data gradients) and the
        # convs in bf16: 0.402-0.404 vs 0.410-0.413 ms/step with the e4m3 convs, bf16 0.409-0.410
        # (profiles/r3_07_fp8_step_variants.txt).
        f8m = getattr(model, "fp8_scales", None)
        self.f8conv = (self.fp8 and dev.type == "cuda" and f8m is not None and f8m.n >= 6
                       and KNOBS.fp8_conv)
        self.f8s, self.f8o = (f8m, 2) if self.f8conv else (None, 0)
        if self.f8conv:
            from .optim import FP8_E4M3_MAX
            for j in range(2):
                self.f8s.set_from_tensor(2 + 2 * j + 1, model.conv_w[j + 1])
                # activations: BN-normalised ReLU outputs; the first step's guess, then the delayed amax
                a = 8.0 * 2.0 ** self.f8s.margin / FP8_E4M3_MAX
                self.f8s.scale[2 + 2 * j] = a
                self.f8s.qs[2 + 2 * j] = 1.0 / a
        self.st = [torch.zeros(U, EC, NST, device=dev) for _ in range(3)]
        # the forward on conv3x3_split_kernel (KNOBS.conv_fwd_split): sps samples per workgroup; its workgroups per group
        # (chunks_f) are the statistics partial rows every BN consumer sums
        self.fwd_split = bool(KNOBS.conv_fwd_split) and not self.f8conv
        self.sps = max(1, int(KNOBS.conv_sps))
        self.chunks_f = (B + self.sps - 1) // self.sps if self.fwd_split else self.chunks
        # layer 1 alone on the split kernel at 4 spw samples per workgroup: conv3x3_kernel's chunking (KNOBS.conv_l1_split)
        self.l1_split = bool(KNOBS.conv_l1_split) and not self.fwd_split and 4 * spw == 12
        self.stats = [torch.zeros(U, self.chunks_f, EC, 2, device=dev) for _ in range(3)]   # per layer
        # BN backward partials per layer, planar rows [sum g | sum g*xhat] x EC (their column sums are
        # dbeta / dgamma: jobs of the step's batched slab reduction)
        # (layers 1, 2: produced by the next layer's fused backward / dgrad kernel, chunked like it;
        # layer 3: by its own reduction launch over dh3 from the FC GEMM)
        self.fuse_bn_red = dx_bf16
        if self.bwd_fused:
            self.rchunks = [self.chunks_wl[1], self.chunks_wl[2], self.chunks_r]
        else:
            self.rchunks = [self.chunks if self.fuse_bn_red else self.chunks_r] * 2 + [self.chunks_r]
        self.rslab = [torch.zeros(U, c, 2, EC, device=dev) for c in self.rchunks]
        # grads w.r.t. h1, h2: bf16 by default (they only feed bf16 MFMA operands and fp32-accumulated
        # BN reductions), halving the dgrad write and every re-read of it
        self.dx_bf16 = dx_bf16
        self.dx = [torch.empty(N, EC, HW, device=dev, dtype=bf if dx_bf16 else torch.float32) for _ in range(2)]
        self.wslab = [torch.empty(self.E, U * c, 32 * cin * 9, device=dev) for c, cin in zip(self.chunks_wl, (2, 32, 32))]
        # bf16 B-fragment images of the weights (re-packed every step; 16-byte coalesced loads in-kernel)
        self.cins = (2, 32, 32)
        self.wpk = [torch.empty(self.E, (9 * cin + 15) // 16, 64, 8, device=dev, dtype=bf) for cin in self.cins]
        self.wpk_t = [None] + [torch.empty(self.E, 18, 64, 8, device=dev, dtype=bf) for _ in range(2)]
        self.lib = nat.hip_lib()
        L = self.lib
        self._fwd = nat.fn(L, "qd_conv_fwd", [_i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p])
        # layers 2 / 3 at P128: the software-pipelined forward (two LDS tiles per wave; bit-identical outputs)
        self._fwd_db = nat.fn(L, "qd_conv_fwd_db", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p])
        self._fwd_split = nat.fn(L, "qd_conv_fwd_split", [_i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p])
        self.fwd_db = bool(KNOBS.conv_fwd_db) and self.W == 8 and self.H == 16
        self._dgrad = nat.fn(L, "qd_conv_dgrad", [_p, _i, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p])
        self._wgrad = nat.fn(L, "qd_conv_wgrad", [_i, _p, _p, _p, _i, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p])
        self._fin = nat.fn(L, "qd_bn_stats_finalize_multi", [_i, _p, _p, _p, _p, _p, _p, _i, _i, _i, _f, _f, _f, _i,
                                                                _p, _i, ctypes.c_longlong, _p])
        self._bred = nat.fn(L, "qd_bn_bwd_reduce", [_p, _i, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p])
        self._bfin = nat.fn(L, "qd_bn_bwd_finalize", [_p, _p, _p, _p, _p, _i, _i, _i, _f, _i, _p])
        self._apply = nat.fn(L, "qd_bn_relu_apply", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p])
        self._apply_tail = nat.fn(L, "qd_bn_apply_tail", [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i,
                                                           _i, _p, _i, ctypes.c_longlong, _p, _p, _p, _p])
        # the BN tail (running statistics) and layer 3's BN/ReLU apply as ONE launch (False: two launches, the
        # tail publishing layer 3's records -- 1 launch more on the chain)
        self.apply_tail = True
        self.spb_a = 8   # (samples per BN-apply workgroup; a group's last workgroup may be partial)
        self._packm = nat.fn(L, "qd_conv_pack_weights_multi", [_i, _p, _p, _p, _p, _i, _p])
        self._packm2 = nat.fn(L, "qd_conv_pack_weights_multi2", [_i, _p, _p, _p, _p, _i, _p, _i, _p])
        # pack_at_tail: the owner packs the weights at the END of each step (after the optimizer) and
        # the forward reads the packed images as they are (one launch less at the head of the chain)
        self.pack_at_tail = False
        self._wd = nat.fn(L, "qd_conv_wgrad_dgrad", [_p, _p, _p, _p, _p, _p, _i, _i, _p, _p, _i, _i, _i, _i, _i, _i, _i,
                                                        _p, _p, _p])
        # (bwd_fused off) wgrad + dgrad of layers 3 and 2 as one launch each
        self.fuse_wd = True
        self._bwdf = nat.fn(L, "qd_conv_bwd_db" if self.bwd_db else "qd_conv_bwd_fused", [_p] * 9 + [_i] * 7 + [_p, _p, _p])
        # layer 3's BN backward partials from the FC data gradient's epilogue (enable_dgrad_bnred): 0 = own launch
        self.bnred_mt = 0
        self._fwd8 = nat.fn(L, "qd_conv_fwd_f8", [_p] * 4 + [_i] * 7 + [_p] * 6)
        # the training forward as ONE persistent launch (conv_fwd_stack_kernel: the 3 layers + the BN tail, per-stream
        # barriers between layers) when its grid fits the chip at once; the bf16 FC operand only (the fp8
        # estimator's e4m3 copy and amax come from the per-layer path's BN tail)
        self.stack = bool(KNOBS.conv_stack and dev.type == "cuda" and not self.fp8 and not self.f8conv
                          and not self.fwd_split
                          and nat.fn(L, "qd_conv_fwd_stack_fits", [_i] * 6)(self.N, self.E, self.B, self.H, self.W,
                                                                           self.chunks))
        if self.stack:
            self._stackf = nat.fn(L, "qd_conv_fwd_stack", [_p, _p] + [_i] * 7 + [_p])
            # barriers (U*E x 2), per-(expert, layer) arrival counts (E x 3), the error word: zero between launches
            self.stack_sync = torch.zeros(2 * U * self.E + 3 * self.E + 1, dtype=torch.int32, device=dev)

    def enable_dgrad_bnred(self, mt: int) -> None:
        """Layer 3's BN backward partials come from the FC data gradient's epilogue (ops.fc.gemm_dgrad_bnred,
        ``mt`` M tiles: partial rows (U, mt, 2, EC); rows of (group, tile) pairs that share no sample stay zero
        from here), so backward() launches no reduction for layer 3 and hands the deferred loss finish to layer
        3's fused backward kernel.  Needs the fused backward (bf16 dx)."""
        assert self.bwd_fused and self.E == 3
        self.bnred_mt = int(mt)
        self.rchunks[2] = self.bnred_mt
        self.rslab[2] = torch.zeros(self.U, self.bnred_mt, 2, self.EC, device=self.rslab[2].device)

    def pack_weights(self, st, cursor: Optional[torch.Tensor] = None, cursor_inc: int = 0) -> None:
        """Forward (3) and dgrad (2) B-fragment images of the current weights: one launch.
        ``cursor`` (int32 device, optional): advanced by ``cursor_inc`` in the same launch."""
        jobs = [(k, 0) for k in range(3)] + [(k, 1) for k in (1, 2)]
        w = (ctypes.c_void_p * 8)(*[nat.ptr(self.m.conv_w[k]) for k, _ in jobs])
        out = (ctypes.c_void_p * 8)(*[nat.ptr(self.wpk_t[k] if d else self.wpk[k]) for k, d in jobs])
        cin = (ctypes.c_int * 8)(*[self.cins[k] for k, _ in jobs])
        dg = (ctypes.c_int * 8)(*[d for _, d in jobs])
        nat.check(self._packm2(len(jobs), w, out, cin, dg, self.E, _ptr(cursor), int(cursor_inc), st),
                  "conv_pack_weights")

    def pack_scatter(self, flat: torch.Tensor, lo: int, hi: int, cursor: Optional[torch.Tensor] = None,
                     cursor_inc: int = 0):
        """PackScatter for an optimizer launch over flat[lo:hi]: the update kernel writes the forward
        (3 layers) and dgrad (layers 2, 3) images of the conv weights it updates -- the same bytes as
        pack_weights -- and advances ``cursor``.  The images' zero padding comes from pack_weights (init)."""
        from .optim import PackScatter
        ps = PackScatter()
        base = flat.data_ptr()
        for k in range(3):
            w = self.m.conv_w[k]
            o = (w.data_ptr() - base) // 4
            if lo <= o and o + w.numel() <= hi:
                ps.lo[k], ps.n[k], ps.cin[k] = o - lo, w.numel(), self.cins[k]
                ps.fwd[k] = nat.ptr(self.wpk[k])
                ps.dg[k] = nat.ptr(self.wpk_t[k]) if self.wpk_t[k] is not None else None
        ps.cursor = nat.ptr(cursor) if cursor is not None else None
        ps.cursor_inc = int(cursor_inc)
        return ps

    # --------------------------------------------------------------------- forward
    def forward(self, x1: torch.Tensor, training: bool) -> torch.Tensor:
        """x1: (N, E*2, H, W) fp32 contiguous.  Returns the FC operand (N*E, 32*H*W) bf16."""
        m, st = self.m, nat.stream_ptr(x1.device)
        assert x1.shape == (self.N, 2 * self.E, self.H, self.W) and x1.dtype == torch.float32 and x1.is_contiguous()
        self.x1 = x1
        if not self.pack_at_tail:
            self.pack_weights(st)
        hook = self.stage_hook
        if hook is not None:
            hook("packed")
        if training and self.stack:
            self._forward_stack(x1, st)
            if hook is not None:
                for k in range(3):
                    hook(f"conv{k + 1}")
            return self.h3
        f8 = self.f8s
        inp, st_prev = x1, None
        for k in range(3):
            # layers 2, 3 finalise the previous layer's BatchNorm themselves (BnFwd: statistics
            # partials -> records, running stats, published st); layer 3's own BN keeps a launch
            bnf = None
            if k > 0:
                j = k - 1
                bnf = BnFwd(nat.ptr(self.stats[j]), nat.ptr(m.bn_w[j]), nat.ptr(m.bn_b[j]), nat.ptr(m.run_mean[j]),
                            nat.ptr(m.run_var[j]), nat.ptr(self.st[j]), self.chunks_f, float(self.B * self.HW),
                            m.momentum, m.eps, int(training))
            if self.l1_split and k == 0:
                nat.check(self._fwd_split(1, nat.ptr(inp), None, nat.ptr(self.wpk[0]), nat.ptr(self.z[0]),
                                          nat.ptr(self.stats[0]), self.N, self.E, self.B, self.H, self.W, self.chunks,
                                          12, None, st), "conv_fwd_split1")
            elif self.fwd_split:
                nat.check(self._fwd_split(k + 1, nat.ptr(inp), _ptr(st_prev), nat.ptr(self.wpk[k]), nat.ptr(self.z[k]),
                                          nat.ptr(self.stats[k]), self.N, self.E, self.B, self.H, self.W, self.chunks_f,
                                          self.sps, ctypes.byref(bnf) if bnf is not None else None, st),
                          f"conv_fwd_split{k + 1}")
            elif self.f8conv and k > 0:
                j = 2 + 2 * (k - 1)
                nat.check(self._fwd8(nat.ptr(inp), nat.ptr(m.conv_w[k]), nat.ptr(self.z[k]), nat.ptr(self.stats[k]),
                                     self.N, self.E, self.B, self.H, self.W, self.chunks, self.spw, ctypes.byref(bnf),
                                     nat.ptr(f8.qs[j:]), nat.ptr(f8.scale[j:]), nat.ptr(f8.amax[j]),
                                     nat.ptr(f8.amax[j + 1]), st), f"conv_fwd_f8_{k + 1}")
            elif k > 0 and self.fwd_db:
                nat.check(self._fwd_db(nat.ptr(inp), _ptr(st_prev), nat.ptr(self.wpk[k]), nat.ptr(self.z[k]),
                                       nat.ptr(self.stats[k]), self.N, self.E, self.B, self.H, self.W, self.chunks,
                                       self.spw, ctypes.byref(bnf) if bnf is not None else None, st),
                          f"conv_fwd_db{k + 1}")
            else:
                nat.check(self._fwd(k + 1, nat.ptr(inp), _ptr(st_prev), nat.ptr(self.wpk[k]), nat.ptr(self.z[k]),
                                    nat.ptr(self.stats[k]), self.N, self.E, self.B, self.H, self.W, self.chunks,
                                    self.spw, ctypes.byref(bnf) if bnf is not None else None, st), f"conv_fwd{k + 1}")
            inp, st_prev = self.z[k], self.st[k]
            if hook is not None:
                hook(f"conv{k + 1}")
        # one BN tail launch: every layer's running statistics (+ num_batches_tracked), and the last
        # layer's records (layers 1, 2 were built -- bitwise identically -- by their consumers)
        nbt = getattr(m, "_nbt", None) if (training and self.count_batches) else None
        arr = lambda xs: (ctypes.c_void_p * 3)(*[nat.ptr(x) for x in xs])
        f8 = self.m.fp8_scales if self.fp8 else None
        if self.apply_tail:
            bnf3 = BnFwd(nat.ptr(self.stats[2]), nat.ptr(m.bn_w[2]), nat.ptr(m.bn_b[2]), nat.ptr(m.run_mean[2]),
                         nat.ptr(m.run_var[2]), nat.ptr(self.st[2]), self.chunks_f, float(self.B * self.HW),
                         m.momentum, m.eps, int(training))
            nat.check(self._apply_tail(nat.ptr(self.z[2]), nat.ptr(self.h3), ctypes.byref(bnf3), arr(self.stats),
                                       arr(m.bn_w), arr(m.bn_b), arr(m.run_mean), arr(m.run_var), arr(self.st),
                                       self.U, self.E, self.B, self.HW, self.spb_a, self.chunks_f, int(training),
                                       _ptr(nbt), nbt.numel() if nbt is not None else 0, self.U, _ptr(self.h3_8),
                                       nat.ptr(f8.qs) if f8 else None, nat.ptr(f8.amax[0]) if f8 else None, st),
                      "bn_apply_tail")
            return self.h3
        nat.check(self._fin(3, arr(self.stats), arr(m.bn_w), arr(m.bn_b), arr(m.run_mean), arr(m.run_var), arr(self.st),
                            self.U, self.chunks_f, self.EC, float(self.B * self.HW), m.momentum, m.eps, int(training),
                            _ptr(nbt), nbt.numel() if nbt is not None else 0, self.U, st), "bn_tail")
        nat.check(self._apply(nat.ptr(self.z[2]), nat.ptr(self.st[2]), nat.ptr(self.h3), self.N, self.EC, self.B,
                              self.HW, _ptr(self.h3_8), nat.ptr(f8.qs) if f8 else None,
                              nat.ptr(f8.amax[0]) if f8 else None, st), "bn_relu_apply")
        return self.h3

    def _forward_stack(self, x1: torch.Tensor, st) -> None:
        a = self.stack_args(x1)
        nat.check(self._stackf(ctypes.byref(a), nat.ptr(self.stack_sync), self.N, self.E, self.B, self.H, self.W,
                               self.chunks, self.spw, st), "conv_fwd_stack")

    def stack_args(self, x1: torch.Tensor) -> "StackFwd":
        """The persistent forward's operand struct for input ``x1`` (also the stamped diagnostic's)."""
        m = self.m
        nbt = getattr(m, "_nbt", None) if self.count_batches else None
        assert nbt is None or nbt.numel() == 3 * self.E, "num_batches_tracked: 3 counters per expert"
        a = StackFwd()
        a.x1 = nat.ptr(x1)
        for k in range(3):
            a.w[k], a.z[k], a.stats[k] = nat.ptr(self.wpk[k]), nat.ptr(self.z[k]), nat.ptr(self.stats[k])
            a.gamma[k], a.beta[k] = nat.ptr(m.bn_w[k]), nat.ptr(m.bn_b[k])
            a.run_mean[k], a.run_var[k], a.st[k] = nat.ptr(m.run_mean[k]), nat.ptr(m.run_var[k]), nat.ptr(self.st[k])
        a.h3 = nat.ptr(self.h3)
        a.nbt = _ptr(nbt)
        a.nbt_inc = self.U
        a.count, a.momentum, a.eps = float(self.B * self.HW), float(m.momentum), float(m.eps)
        return a

    def stack_error(self) -> bool:
        """True when a persistent forward's barrier wait gave up (its outputs are then wrong): callers check it at
        a synchronisation point (bench / epoch end)."""
        return bool(self.stack and int(self.stack_sync[-1]) != 0)

    # --------------------------------------------------------------------- backward
    def backward(self, dh3: torch.Tensor, accumulate: bool = True, slabs: Optional["SlabBatch"] = None,
                 side: Optional["torch.cuda.Stream"] = None, loss_finish=None) -> None:
        """dh3: dL/dh3 as (N*E, 32*H*W) (bf16 or fp32).  Adds (accumulate) or writes the conv/BN grads
        into the flat grad -- writing makes a zero_grad before the step unnecessary.

        ``side``: a second stream for the weight-gradient kernels of layers 3 and 2.  wgrad(k) and
        dgrad(k) only share their inputs, so the dgrad chain (the critical path to layer 1) runs on
        the current stream while wgrad(k) runs beside it; the current stream joins before the slab
        reduction.  Each of these kernels fills well under the 256 CUs, so they overlap.
        ``loss_finish`` (ops.nmse.LossFinish): the deferred HDCE loss finish, hosted by layer 3's BN
        reduction launch as one extra workgroup (with ``bnred_mt``: by layer 3's fused backward launch)."""
        m, st = self.m, nat.stream_ptr(dh3.device)
        main = torch.cuda.current_stream(dh3.device) if side is not None else None
        dh, dh_bf = dh3, int(dh3.dtype == torch.bfloat16)
        side_used = False
        for k in (2, 1, 0):
            z, bst = self.z[k], self.st[k]
            rs = self.rslab[k]
            lf = ctypes.byref(loss_finish) if (loss_finish is not None and k == 2) else None
            # (layer 3 with bnred_mt: the FC data gradient's epilogue produced them; else the previous dgrad)
            if (k == 2 and not self.bnred_mt) or (k < 2 and not self.fuse_bn_red):
                nat.check(self._bred(nat.ptr(dh), dh_bf, nat.ptr(z), nat.ptr(bst), nat.ptr(rs), self.N, self.E,
                                     self.B, self.H, self.W, self.chunks_r, self.spb_r, lf, st), f"bn_bwd_reduce{k + 1}")
                lf = None
            # BN backward finalisation fused into this layer's wgrad and dgrad kernels
            bnb = BnBwd(nat.ptr(rs), nat.ptr(m.bn_w[k]), self.rchunks[k], float(self.B * self.HW))
            xin = self.x1 if k == 0 else self.z[k - 1]
            st_prev = None if k == 0 else self.st[k - 1]
            ws = self.wslab[k]
            # (the fused kernel has no separate weight-gradient launch to put on ``side``)
            if k > 0 and self.bwd_fused and dh_bf:
                dx = self.dx[k - 1]
                nat.check(self._bwdf(nat.ptr(xin), _ptr(st_prev), nat.ptr(dh), nat.ptr(z), nat.ptr(bst), nat.ptr(ws),
                                     nat.ptr(self.wpk_t[k]), nat.ptr(dx), nat.ptr(self.rslab[k - 1]), self.N, self.E,
                                     self.B, self.H, self.W, self.chunks_wl[k], self.spb_wl[k], ctypes.byref(bnb), lf,
                                     st), f"conv_bwd_fused{k + 1}")
                dh, dh_bf = dx, 1
                continue
            assert lf is None, "the deferred loss finish needs layer 3's fused backward launch"
            if k > 0 and self.fuse_wd and dh_bf and self.dx_bf16 and side is None:
                # weight AND data gradient of this layer in one launch (independent: side by side)
                dx = self.dx[k - 1]
                brd = BnRed(nat.ptr(self.z[k - 1]), nat.ptr(self.st[k - 1]), nat.ptr(self.rslab[k - 1])) \
                    if self.fuse_bn_red else None
                nat.check(self._wd(nat.ptr(xin), _ptr(st_prev), nat.ptr(dh), nat.ptr(z), nat.ptr(bst), nat.ptr(ws),
                                   self.chunks_wl[k], self.spb_wl[k], nat.ptr(self.wpk_t[k]), nat.ptr(dx), self.chunks,
                                   self.spw, self.N, self.E, self.B, self.H, self.W, ctypes.byref(bnb),
                                   ctypes.byref(brd) if brd is not None else None, st), f"conv_wgrad_dgrad{k + 1}")
                dh, dh_bf = dx, 1
                continue
            on_side = side is not None and k > 0
            if on_side:
                side.wait_stream(main)
                side_used = True
            wst = nat.stream_ptr(dh3.device) if not on_side else ctypes.c_void_p(side.cuda_stream)
            nat.check(self._wgrad(k + 1, nat.ptr(xin), _ptr(st_prev), nat.ptr(dh), dh_bf, nat.ptr(z), nat.ptr(bst),
                                  nat.ptr(ws), self.N, self.E, self.B, self.H, self.W, self.chunks_wl[k], self.spb_wl[k],
                                  ctypes.byref(bnb), wst), f"conv_wgrad{k + 1}")
            if k > 0:
                dx = self.dx[k - 1]
                # ... and the previous layer's BN backward reduction fused into this dgrad's epilogue
                brd = BnRed(nat.ptr(self.z[k - 1]), nat.ptr(self.st[k - 1]), nat.ptr(self.rslab[k - 1])) \
                    if self.fuse_bn_red else None
                nat.check(self._dgrad(nat.ptr(dh), dh_bf, nat.ptr(z), nat.ptr(bst), nat.ptr(self.wpk_t[k]),
                                      nat.ptr(dx), int(self.dx_bf16), self.N, self.E, self.B, self.H, self.W,
                                      self.chunks, self.spw, ctypes.byref(bnb),
                                      ctypes.byref(brd) if brd is not None else None, st), f"conv_dgrad{k + 1}")
                dh, dh_bf = dx, int(self.dx_bf16)
        if side_used:
            main.wait_stream(side)
        # the three weight-gradient slabs -> conv_w grads: queued on the caller's batch (one launch
        # for every slab reduction of the step phase) or launched here
        own = slabs is None
        batch = SlabBatch() if own else slabs
        EC = self.EC
        for k in range(3):
            w = self.wslab[k]
            R = self.U * self.rchunks[k]
            batch.add(w, m.conv_w[k].grad, self.E, w.shape[1], w.shape[2])
            batch.add(self.rslab[k], m.bn_b[k].grad, 1, R, EC, ld=2 * EC)              # dbeta = sum g
            batch.add(self.rslab[k], m.bn_w[k].grad, 1, R, EC, ld=2 * EC, offset=EC)   # dgamma = sum g*xhat
        if own:
            batch.launch(accumulate, st)
