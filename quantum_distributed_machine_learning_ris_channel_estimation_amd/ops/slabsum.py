"""Batched deterministic gradient-slab reductions (csrc/hip/conv.hip ``qd_slab_rows_sum_multi``).

Several fused backward kernels (conv weight gradients, the quantum layer's adjoint pass, the QSC
preprocess backward) write per-workgroup partial rows ("slabs") instead of using float atomics;
each slab is summed over its rows into the flat gradient buffer.  Every such reduction of a step
phase is independent, so ``SlabBatch`` collects them and issues ONE launch (up to 8 jobs) -- on
this GPU a dependent launch costs ~5 us however little it computes.
"""
from __future__ import annotations

import ctypes
from typing import List, Tuple

import torch

from .. import _native as nat

_p, _i = ctypes.c_void_p, ctypes.c_int
MAX_JOBS = 16


class SlabBatch:
    def __init__(self):
        self.jobs: List[Tuple[int, torch.Tensor, int, int, int, int]] = []
        self._f = None

    def add(self, slab: torch.Tensor, out: torch.Tensor, groups: int, rows: int, width: int, ld: int = 0,
            offset: int = 0) -> None:
        """out[g, :width] (+)= sum_r slab[offset + (g * rows + r) * ld : ... + width] for g < groups
        (fp32; ld = row stride, default width)."""
        ld = ld or width
        assert slab.dtype == torch.float32 and out.dtype == torch.float32 and slab.is_contiguous()
        assert offset + (groups * rows - 1) * ld + width <= slab.numel() and out.numel() >= groups * width
        if len(self.jobs) == MAX_JOBS:
            raise RuntimeError(f"SlabBatch: more than {MAX_JOBS} reductions in one launch")
        self.jobs.append((slab.data_ptr() + 4 * offset, out, groups, rows, width, ld))

    def jobs_in(self, flat_grad: torch.Tensor, lo: int, hi: int):
        """The queued reductions as slab jobs of an optimizer launch over flat_grad[lo:hi] (ops/optim.py
        ``step(slabs=...)``): (slab pointer, offset relative to lo, groups, rows, width, ld) per job.  Every output
        must be a float32 view into flat_grad[lo:hi], and the whole batch is consumed (nothing is launched here)."""
        base = flat_grad.data_ptr()
        out = []
        for slab_ptr, o, groups, rows, width, ld in self.jobs:
            off = (o.data_ptr() - base) // 4
            if o.dtype != torch.float32 or (o.data_ptr() - base) % 4 or off < lo or off + groups * width > hi:
                raise ValueError("slab job output outside the optimizer's range")
            out.append((slab_ptr, off - lo, groups, rows, width, ld))
        self.jobs = []
        return out

    def launch(self, accumulate: bool, stream) -> None:
        if not self.jobs:
            return
        if self._f is None:
            self._f = nat.fn(nat.hip_lib(), "qd_slab_rows_sum_multi", [_i, _p, _p, _p, _p, _p, _p, _i, _p])
        n = len(self.jobs)
        slabs = (ctypes.c_void_p * n)(*[j[0] for j in self.jobs])
        outs = (ctypes.c_void_p * n)(*[nat.ptr(j[1]) for j in self.jobs])
        groups = (ctypes.c_int * n)(*[j[2] for j in self.jobs])
        rows = (ctypes.c_int * n)(*[j[3] for j in self.jobs])
        widths = (ctypes.c_int * n)(*[j[4] for j in self.jobs])
        lds = (ctypes.c_int * n)(*[j[5] for j in self.jobs])
        nat.check(self._f(n, slabs, outs, groups, rows, widths, lds, int(accumulate), stream), "slab_rows_sum_multi")
        self.jobs = []
