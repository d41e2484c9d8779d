"""Flat parameter spaces and the fused optimizers that update them.

Reference optimizers: ``Y2HRunner.get_optimizer`` (Runner_P128_QuantumNAT_onchipQNN.py:40-46),
four separate ``Adam``s for Conv0/1/2 + CE (R:160-163), ``AdamW(wd=0.01)`` for the QSC
(R:320), and ``QSC_P128.apply_gradient_pruning`` (E:205-228).

``FlatParamSpace`` re-points every parameter of a set of modules at a view of ONE
contiguous fp32 buffer (grads likewise), so that
  * zero_grad is one memset,
  * the data-parallel gradient all-reduce is one RCCL call per bucket,
  * the optimizer step is one HIP kernel (csrc/hip/optim.hip) -- four Adams with
    identical hyper-parameters are exactly one Adam over the concatenation.
All step-dependent scalars live on the device, so a captured HIP graph replays
correctly step after step (LR changes are a device write, not a re-capture).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from .. import _native as nat

_p, _i, _f, _l = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_long
ALIGN = 16  # elements; keeps every parameter view 64-byte aligned for float4 access


class PackScatter(ctypes.Structure):
    """csrc/hip/optim.hip ``PackScatter``: conv weight images written by the update kernel itself."""
    _fields_ = [("lo", ctypes.c_long * 3), ("n", ctypes.c_int * 3), ("cin", ctypes.c_int * 3),
                ("fwd", ctypes.c_void_p * 3), ("dg", ctypes.c_void_p * 3), ("cursor", ctypes.c_void_p),
                ("cursor_inc", ctypes.c_int)]


class FlatParamSpace:
    def __init__(self, params: Sequence[Tuple[str, nn.Parameter]], device=None, extra: int = 0, front: int = 0,
                 storage: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
        """``extra``: trailing scratch floats (one ALIGN block) after the last parameter; their grad
        slots ride along with the tail of the grad buffer (e.g. a NaN flag that then travels in the
        same all-reduce as the last parameters' gradients).  ``extra_off`` is their offset.
        ``front``: floats reserved IN FRONT of this space in the same allocation (``front_views``: (flat, grad)
        of that region) -- another space placed there with ``storage`` makes the two gradient buffers one
        contiguous range (one in-place collective, no coalescing copies).  ``storage``: (flat, grad) views to
        live in instead of a fresh allocation (zero-filled by their owner, at least ``size_of`` long)."""
        uniq = self._uniq(params)
        self.names = [n for n, _ in uniq]
        self.params = [p for _, p in uniq]
        device = torch.device(device) if device is not None else self.params[0].device
        offs, off = [], 0
        for p in self.params:
            offs.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.offsets = offs
        self.extra_off = off
        off += (extra + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.n_real = sum(p.numel() for p in self.params)
        self.front_views = None
        if storage is not None:
            if front or storage[0].numel() < off or storage[1].numel() < off:
                raise ValueError(f"storage of {storage[0].numel()} floats for a space of {off}")
            self.flat, self.grad = storage[0][:off], storage[1][:off]
            self.grad_base = None
        else:
            if front % ALIGN:
                raise ValueError(f"front {front} not a multiple of {ALIGN}")
            fa = torch.zeros(front + off, device=device, dtype=torch.float32)
            ga = torch.zeros(front + off, device=device, dtype=torch.float32)
            self.flat, self.grad = fa[front:], ga[front:]
            self.grad_base = ga   # (front region + this space's gradients, contiguous)
            if front:
                self.front_views = (fa[:front], ga[:front])
        for p, o in zip(self.params, offs):
            n = p.numel()
            view = self.flat[o:o + n].view(p.shape)
            view.copy_(p.data.to(device, torch.float32))
            p.data = view
            p.grad = self.grad[o:o + n].view(p.shape)

    @staticmethod
    def _uniq(params):
        seen, uniq = set(), []
        for name, p in params:
            if id(p) in seen:
                continue
            seen.add(id(p))
            uniq.append((name, p))
        return uniq

    @classmethod
    def size_of(cls, params: Sequence[Tuple[str, nn.Parameter]], extra: int = 0) -> int:
        """Floats a space over ``params`` (+ ``extra``) occupies (shapes only: meta tensors will do)."""
        al = lambda n: (n + ALIGN - 1) // ALIGN * ALIGN
        return sum(al(p.numel()) for _, p in cls._uniq(params)) + al(extra)

    def slice_of(self, p: torch.Tensor) -> slice:
        for q, o in zip(self.params, self.offsets):
            if q is p:
                return slice(o, o + q.numel())
        raise KeyError("parameter not in space")

    def zero_grad(self) -> None:
        self.grad.zero_()

    def reattach_grads(self) -> None:
        """Restore the grad views if user code set ``p.grad = None``."""
        for p, o in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:].data_ptr():
                p.grad = self.grad[o:o + p.numel()].view(p.shape)


FP8_E4M3_MAX = 448.0


class Fp8Scales:
    """Delayed per-tensor fp8 scaling state for ``n`` tensors (device-resident, graph-safe).

    ``qs[i]`` is the quantisation factor producers multiply by (x8 = e4m3(x * qs)), ``scale[i]`` =
    1/qs the dequantisation factor handed to the GEMM, ``amax[i]`` the per-workgroup max |x|
    partials the producers write (no atomics); ``update()`` (one launch) reduces them into the
    next scales and re-arms them."""

    PARTS = 4096   # = kAmaxParts in csrc/hip/common.h

    def __init__(self, n: int, device, margin: float = 1.0):
        self.n, self.margin = n, margin
        self.amax = torch.zeros(n, self.PARTS, device=device, dtype=torch.float32)
        if self.amax.is_cuda:
            assert nat.fn(nat.hip_lib(), "qd_amax_parts", [])() == self.PARTS
        self.scale = torch.ones(n, device=device, dtype=torch.float32)
        self.qs = torch.ones(n, device=device, dtype=torch.float32)

    def set_from_tensor(self, i: int, t: torch.Tensor) -> None:
        a = float(t.detach().abs().max().clamp_min(1e-30))
        s = a * 2.0 ** self.margin / FP8_E4M3_MAX
        self.scale[i] = s
        self.qs[i] = 1.0 / s

    def update(self) -> None:
        if self.scale.is_cuda:
            f = nat.fn(nat.hip_lib(), "qd_fp8_scale_update", [_p, _p, _p, _i, _f, _f, _p])
            nat.check(f(nat.ptr(self.amax), nat.ptr(self.scale), nat.ptr(self.qs), self.n, FP8_E4M3_MAX,
                        self.margin, nat.stream_ptr(self.scale.device)), "fp8_scale_update")
            return
        a = self.amax.amax(dim=1)
        upd = a > 0
        s = a.clamp_min(1e-30) * 2.0 ** self.margin / FP8_E4M3_MAX
        self.scale.copy_(torch.where(upd, s, self.scale))
        self.qs.copy_(1.0 / self.scale)
        self.amax.zero_()


class FusedOptimizer:
    """Adam / AdamW / SGD-momentum over a FlatParamSpace, one kernel per step.

    ``prune_thr`` > 0 fuses on-chip gradient pruning (g *= |g| > thr) into the step,
    ``grad_scale`` fuses gradient averaging; ``skip`` (device fp32, nonzero = skip) makes the step a no-op.
    """

    def __init__(self, space: FlatParamSpace, kind: str = "adam", lr: float = 1e-3, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, momentum: float = 0.9, prune_thr: float = 0.0):
        if kind not in ("adam", "adamw", "sgd"):
            raise NotImplementedError(f"Optimizer {kind} not understood.")
        self.space = space
        self.kind = kind
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.momentum = momentum
        self.prune_thr = prune_thr
        dev = space.flat.device
        self.lr_t = torch.full((1,), lr, device=dev, dtype=torch.float32)
        # parts: [lo, hi) ranges of the flat space stepped by separate launches (``step(part=i)``), each
        # with its own step counter / done counter, so independent ranges can update on different
        # streams as soon as their gradients are final (they always advance together: equal counts)
        self.bounds: List[Tuple[int, int]] = [(0, space.numel)]
        self.end = space.numel   # stepped range ends here (limit())
        self.max_grid: Dict[int, int] = {}   # part -> workgroup cap of its update launch (0: default)
        self.step_t = torch.zeros(1, device=dev, dtype=torch.float32)
        self.pruned = torch.zeros(1, device=dev, dtype=torch.int32)
        self.done = torch.zeros(1, device=dev, dtype=torch.int32)   # last-workgroup counter (step tick)
        self.shadow: Optional[torch.Tensor] = None                    # bf16 copy of flat[lo:hi]
        self.shadow_lo = self.shadow_hi = 0
        self.shadow8: Optional[torch.Tensor] = None                   # e4m3 copy (fp8 estimator)
        self.fp8: Optional[Fp8Scales] = None
        self.fp8_slot = 0
        if kind == "sgd":
            self.buf = torch.zeros_like(space.flat)
        else:
            self.m = torch.zeros_like(space.flat)
            self.v = torch.zeros_like(space.flat)
        self._lr_host = lr
        # (GPU) a range [lo, hi) stepped by ANOTHER kernel (the FC weight, inside its weight-gradient GEMM's
        # epilogue, ops/fc.gemm_wgrad_adam): every launch here skips it; it has its own step / done slot
        self.fused: Optional[Tuple[int, int]] = None
        # torch.optim-like view for code that reads/writes param_groups[0]['lr']
        self.param_groups = [_LRGroup(self)]

    def partition(self, cuts: Sequence[int]) -> None:
        """Split the space at the (ALIGN-multiple) offsets ``cuts`` into independently launched parts."""
        edges = [0] + sorted(int(c) for c in cuts) + [self.end]
        if any(e % 4 for e in edges) or any(a >= b for a, b in zip(edges, edges[1:])):
            raise ValueError(f"bad partition {edges}")
        self.bounds = list(zip(edges, edges[1:]))
        dev = self.space.flat.device
        self.step_t = self.step_t[:1].repeat(len(self.bounds)).contiguous()
        self.done = torch.zeros(len(self.bounds), device=dev, dtype=torch.int32)

    def limit(self, end: int) -> None:
        """Step nothing at or past ``end`` (an ALIGN-multiple offset): the space's trailing scratch there holds
        flags that other kernels read while this optimizer runs (the DP plan's NaN flags ride in the gradient
        buckets), and a step would rewrite them in place (grad_scale / pruning write the gradient back) and
        count them in the pruning statistics."""
        if end % 4 or end <= 0 or end > self.space.numel:
            raise ValueError(f"limit {end} for a space of {self.space.numel}")
        if self.bounds[-1][0] >= end:
            raise ValueError(f"limit {end} would empty the last part {self.bounds[-1]}")
        self.bounds = [(lo, min(hi, end)) for lo, hi in self.bounds if lo < end]
        self.end = end

    def fuse_range(self, lo: int, hi: int) -> int:
        """Hand [lo, hi) (inside ONE part) to an external update kernel; returns the index of its step / done
        slot (step_t[i], done[i]).  GPU only; Adam without weight decay or pruning, no e4m3 shadow."""
        if not self.space.flat.is_cuda or self.kind != "adam" or self.weight_decay or self.prune_thr or self.fp8:
            raise ValueError("fused ranges: GPU Adam (no weight decay / pruning / e4m3 shadow) only")
        if lo % 4 or hi % 4 or not any(a <= lo and hi <= b for a, b in self.bounds):
            raise ValueError(f"fused range {(lo, hi)} must be 4-aligned and inside one part of {self.bounds}")
        self.fused = (lo, hi)
        dev = self.space.flat.device
        self.step_t = torch.cat([self.step_t, self.step_t[:1].clone()]).contiguous()
        self.done = torch.cat([self.done, torch.zeros(1, device=dev, dtype=torch.int32)])
        return len(self.bounds)

    def attach_shadow(self, lo: int, hi: int, fp8: Optional[Fp8Scales] = None, fp8_slot: int = 0) -> torch.Tensor:
        """Keep a bf16 copy of flat[lo:hi] up to date with every step (written by the update
        kernel itself on the GPU).  Returns the shadow, initialised from the current weights.
        With ``fp8``, an e4m3 copy (``shadow8``, quantised with fp8.qs[fp8_slot]) is kept too and
        the kernel accumulates max|w| into fp8.amax[fp8_slot]."""
        if lo % 4 or hi % 4:
            raise ValueError("shadow bounds must be multiples of 4")
        self.shadow_lo, self.shadow_hi = lo, hi
        self.shadow = self.space.flat[lo:hi].to(torch.bfloat16)
        if fp8 is not None:
            self.fp8, self.fp8_slot = fp8, fp8_slot
            fp8.set_from_tensor(fp8_slot, self.space.flat[lo:hi])
            self.shadow8 = torch.empty(hi - lo, device=self.space.flat.device, dtype=torch.float8_e4m3fn)
        self.refresh_shadow()
        return self.shadow

    def refresh_shadow(self) -> None:
        """Re-sync the shadow after the weights were changed outside step() (load, broadcast)."""
        if self.shadow is not None:
            w = self.space.flat[self.shadow_lo:self.shadow_hi]
            self.shadow.copy_(w)
            if self.shadow8 is not None:
                q = self.fp8.qs[self.fp8_slot]
                self.shadow8.copy_((w * q).clamp(-FP8_E4M3_MAX, FP8_E4M3_MAX).to(torch.float8_e4m3fn))

    # ---------------------------------------------------------------- lr
    @property
    def lr(self) -> float:
        return self._lr_host

    def set_lr(self, lr: float) -> None:
        self._lr_host = float(lr)
        self.lr_t.fill_(float(lr))

    # ---------------------------------------------------------------- step
    def step(self, grad_scale: float = 1.0, skip: Optional[torch.Tensor] = None, part: Optional[int] = None,
             pack=None, slabs=None) -> None:
        """One optimizer step over every part (``part=None``) or over part ``part`` only.  ``pack`` (GPU):
        a callable (lo, hi) -> PackScatter for the range a launch updates (see ConvStackHIP.pack_scatter).
        ``slabs`` (GPU, one part): an ops.slabsum.SlabBatch whose reductions write gradients of this space -- the
        update sums them itself (optim.hip AdamSlabs) instead of a slab launch before it."""
        s = self.space
        parts = range(len(self.bounds)) if part is None else (part,)
        if not s.flat.is_cuda:
            if slabs is not None:
                raise ValueError("slab-fed updates are a GPU path")
            for i in parts:
                self._step_host(i, grad_scale, skip)
            if self.shadow is not None:
                self.refresh_shadow()
            return
        if slabs is not None and (len(parts) != 1 or self.kind != "adam" and self.kind != "adamw"):
            raise ValueError("slab-fed update: one Adam part per launch")
        for i in parts:
            self._step_part(i, grad_scale, skip, pack, slabs=slabs)

    def step_fused(self, grad_scale: float = 1.0, skip: Optional[torch.Tensor] = None, max_grid: int = 0) -> None:
        """(GPU) one Adam launch over the ``fuse_range`` hole itself, on the current stream, with the hole's own
        step / done slot: the range is then stepped apart from (and concurrently with) the other launches --
        e.g. the FC weight's Adam on a side stream beside the conv backward (FlagshipConfig.fc_adam_side).
        ``max_grid``: workgroup cap (0 = the default 2048)."""
        if self.fused is None:
            raise ValueError("step_fused needs a fuse_range")
        lo, hi = self.fused
        self._step_part(len(self.bounds), grad_scale, skip, None, rng=(lo, hi), max_grid=max_grid)

    def _step_part(self, i: int, grad_scale: float, skip: Optional[torch.Tensor], pack=None, rng=None,
                   max_grid: int = 0, slabs=None) -> None:
        s = self.space
        lo, hi = self.bounds[i] if rng is None else rng
        lib = nat.hip_lib()
        st = nat.stream_ptr(s.flat.device)
        skp = nat.ptr(skip) if skip is not None else None
        sp = lambda t: ctypes.c_void_p(t.data_ptr() + 4 * lo)
        step_p, done_p = nat.ptr(self.step_t[i:]), nat.ptr(self.done[i:])
        if self.kind == "sgd":
            f = nat.fn(lib, "qd_sgd_step", [_p, _p, _p, _l, _p, _p, _p, _f, _f, _f, _p, _p])
            nat.check(f(sp(s.flat), sp(s.grad), nat.ptr(self.buf[lo:]), hi - lo, nat.ptr(self.lr_t), step_p, skp,
                        self.momentum, self.weight_decay, grad_scale, done_p, st), "sgd")
            if self.shadow is not None:
                self.refresh_shadow()
            return
        f = nat.fn(lib, "qd_adam_step_slabs", [_p, _p, _p, _p, _l, _p, _p, _p, _p, _f, _f, _f, _f, _i, _f, _f,
                                               _p, _p, _l, _l, _p, _p, _p, _i, _p, _l, _l,
                                               _i, _p, _p, _p, _p, _p, _p, _p])
        jobs = slabs.jobs_in(s.grad, lo, hi) if slabs is not None else []
        nj = len(jobs)
        col = lambda k, ty: (ty * max(nj, 1))(*[j[k] for j in jobs]) if nj else None
        hole_lo = hole_n = 0
        if rng is None and self.fused is not None and lo <= self.fused[0] and self.fused[1] <= hi:
            hole_lo, hole_n = self.fused[0] - lo, self.fused[1] - self.fused[0]
        ps = pack(lo, hi) if pack is not None else None
        # the shadow range, clipped to this part and expressed relative to it
        sh_lo, sh_hi = max(self.shadow_lo, lo), min(self.shadow_hi, hi)
        has_sh = self.shadow is not None and sh_lo < sh_hi
        f8 = has_sh and self.shadow8 is not None
        sh_ptr = ctypes.c_void_p(self.shadow.data_ptr() + 2 * (sh_lo - self.shadow_lo)) \
            if has_sh else None
        sh8_ptr = ctypes.c_void_p(self.shadow8.data_ptr() + (sh_lo - self.shadow_lo)) if f8 else None
        nat.check(f(sp(s.flat), sp(s.grad), nat.ptr(self.m[lo:]), nat.ptr(self.v[lo:]), hi - lo,
                    nat.ptr(self.lr_t), step_p, skp, nat.ptr(self.pruned), self.betas[0],
                    self.betas[1], self.eps, self.weight_decay, int(self.kind == "adamw"), grad_scale,
                    self.prune_thr, done_p, sh_ptr, (sh_lo - lo) if has_sh else 0, (sh_hi - lo) if has_sh else 0,
                    sh8_ptr, nat.ptr(self.fp8.qs[self.fp8_slot:]) if f8 else None,
                    nat.ptr(self.fp8.amax[self.fp8_slot]) if f8 else None, int(max_grid or self.max_grid.get(i, 0)),
                    ctypes.byref(ps) if ps is not None else None, hole_lo, hole_n,
                    nj, col(0, ctypes.c_void_p), col(1, ctypes.c_long), col(2, ctypes.c_int), col(3, ctypes.c_int),
                    col(4, ctypes.c_int), col(5, ctypes.c_int), st),
                  "adam")

    @torch.no_grad()
    def _step_host(self, i: int, grad_scale: float, skip: Optional[torch.Tensor]) -> None:
        """CPU path for part ``i`` (same math as optim.hip; the CPU has no HIP kernels)."""
        if skip is not None and float(skip.item()) != 0.0:
            return
        s = self.space
        lo, hi = self.bounds[i]
        p, g = s.flat[lo:hi], s.grad[lo:hi]
        if grad_scale != 1.0:
            g.mul_(grad_scale)
        if self.prune_thr > 0:
            mask = g.abs() > self.prune_thr
            self.pruned += (~mask).sum().to(torch.int32)
            g.mul_(mask)
        lr = float(self.lr_t.item())
        if self.kind == "sgd":
            buf = self.buf[lo:hi]
            d = g + self.weight_decay * p if self.weight_decay else g
            if self.step_t[i].item() == 0:
                buf.copy_(d)
            else:
                buf.mul_(self.momentum).add_(d)
            p.sub_(lr * buf)
        else:
            m, v = self.m[lo:hi], self.v[lo:hi]
            t = float(self.step_t[i].item()) + 1.0
            b1, b2 = self.betas
            if self.kind == "adamw":
                p.mul_(1 - lr * self.weight_decay)
                d = g
            else:
                d = g + self.weight_decay * p if self.weight_decay else g
            m.mul_(b1).add_(d, alpha=1 - b1)
            v.mul_(b2).addcmul_(d, d, value=1 - b2)
            denom = (v.sqrt() / (1 - b2 ** t) ** 0.5).add_(self.eps)
            p.addcdiv_(m, denom, value=-lr / (1 - b1 ** t))
        self.step_t[i] += 1

    def zero_grad(self) -> None:
        self.space.zero_grad()

    def pruned_count(self, steps: int) -> int:
        """Pruned gradient elements over ``steps`` steps (alignment padding excluded; syncs)."""
        return int(self.pruned.item()) - (self.end - self.space.n_real) * steps

    def pruning_ratio(self, steps: int) -> float:
        return self.pruned_count(steps) / max(1, self.space.n_real * steps)

    # ---------------------------------------------------------------- state
    def state_dict(self) -> Dict:
        d = {"kind": self.kind, "lr": self._lr_host, "step": self.step_t[:1].cpu(), "betas": self.betas, "eps": self.eps,
             "weight_decay": self.weight_decay, "prune_thr": self.prune_thr}
        if self.kind == "sgd":
            d["buf"] = self.buf.cpu()
        else:
            d["m"], d["v"] = self.m.cpu(), self.v.cpu()
        return d

    def load_state_dict(self, d: Dict) -> None:
        self.refresh_shadow()
        self.set_lr(d["lr"])
        self.step_t.copy_(d["step"].reshape(-1)[:1].expand_as(self.step_t))
        if self.kind == "sgd":
            self.buf.copy_(d["buf"])
        else:
            self.m.copy_(d["m"])
            self.v.copy_(d["v"])


class _LRGroup(dict):
    def __init__(self, opt: FusedOptimizer):
        super().__init__()
        self._opt = opt

    def __getitem__(self, k):
        if k == "lr":
            return self._opt.lr
        return super().__getitem__(k)

    def __setitem__(self, k, v):
        if k == "lr":
            self._opt.set_lr(v)
        else:
            super().__setitem__(k, v)


def make_optimizer(space: FlatParamSpace, name: str, lr: float, **kw) -> FusedOptimizer:
    """Reference ``get_optimizer`` semantics: 'adam' -> Adam(lr), 'sgd' -> SGD(lr, 0.9), 'adamw'."""
    name = name.lower()
    if name == "adam":
        return FusedOptimizer(space, "adam", lr, **kw)
    if name == "adamw":
        return FusedOptimizer(space, "adamw", lr, weight_decay=kw.pop("weight_decay", 0.01), **kw)
    if name == "sgd":
        return FusedOptimizer(space, "sgd", lr, momentum=kw.pop("momentum", 0.9), **kw)
    raise NotImplementedError(f"Optimizer {name} not understood.")
