"""One-launch batch assembly from the HBM-resident dataset (csrc/hip/gather.hip).

Reference: the per-step host-side packing + H2D copies of every stream
(Runner_P128_QuantumNAT_onchipQNN.py:104-108, R:181-199, R:344-346).

``StepGather(E, U, B, H, W)`` owns static buffers (graph-capturable) and, for a shuffled
index vector ``idx`` (B,) over a ``DMLStore``, fills
  x1      (U*B, E*2, H, W)  HDCE grouped-conv input
  xq      (S*B, 2, H, W)    classifier input, stream-major (if ``with_classifier``)
  rowoff  (U*B*E,) int32    store row of every FC output row (labels are read in place)
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from .. import _native as nat

_p, _i, _l = ctypes.c_void_p, ctypes.c_int, ctypes.c_long


class StepGather:
    def __init__(self, E: int, U: int, B: int, H: int, W: int, device, with_classifier: bool = True):
        self.E, self.U, self.B, self.H, self.W = E, U, B, H, W
        self.S = E * U
        dev = torch.device(device)
        self.x1 = torch.empty(U * B, E * 2, H, W, device=dev)
        self.xq = torch.empty(self.S * B, 2, H, W, device=dev) if with_classifier else None
        self.rowoff = torch.empty(U * B * E, device=dev, dtype=torch.int32)
        self.plane = 2 * H * W
        # optional (GPU, HDCE half): per-row label / perf powers of the store (rowoff's row space); the
        # cursor gather then also writes rowden (U*B*E, 2) for the one-pass NMSE's denominators
        self.rowpow = None
        self.rowden = torch.zeros(U * B * E, 2, device=dev)
        # strong scaling (the reference's DataParallel split, R:144-148): this rank's part of a global batch of
        # ``adv`` rows per stream starts ``off`` rows in; the cursor advances by adv.  ``den_scale``: per stream
        # (global / part) label powers, so the NMSE sums over this part ARE the global batch's denominators.
        self.off, self.adv = 0, B
        self.den_scale = None
        self.den_global = None   # (S, 2): the global batch's per-stream label / perf powers (the torch NMSE's form)

    def set_part(self, off: int, global_batch: int) -> None:
        """(strong scaling) take rows [off, off + B) of every global batch of ``global_batch`` rows per stream."""
        if off < 0 or off + self.B > global_batch:
            raise ValueError(f"part [{off}, {off + self.B}) of a {global_batch}-row global batch")
        self.off, self.adv = off, global_batch
        if global_batch != self.B:
            self.den_scale = torch.ones(self.S, 2, device=self.rowden.device)
            self.den_global = torch.zeros(self.S, 2, device=self.rowden.device)

    def from_cursor(self, store, perm: torch.Tensor, cursor: torch.Tensor, done: Optional[torch.Tensor],
                    hdce: bool = True, classifier: bool = True) -> None:
        """Batch ``perm[*cursor : *cursor + B]`` (device cursor, int32 (1,)), then ``*cursor += B`` -- all
        in the one launch, so the batch selection is part of a captured graph.  ``hdce`` fills x1 and
        rowoff, ``classifier`` fills xq (two graphs on two streams each gather their half with their
        own cursor).  ``done``: int32 (1,) zero-initialised scratch (last-workgroup counter); None = only
        READ the cursor (the caller advances it later in the step)."""
        Yp, HL = store.Yp, store.Hlabel
        assert perm.dtype == torch.int64 and cursor.dtype == torch.int32
        assert done is None or done.dtype == torch.int32
        cols = HL.shape[-1]
        if Yp.is_cuda:
            assert Yp.dtype == torch.float32 and Yp[0, 0].is_contiguous() and Yp.stride(1) == self.plane
            assert HL.stride(1) == cols and HL.stride(0) % cols == 0 and store.Hperf.stride() == HL.stride()
            assert perm.numel() == Yp.shape[1]
            f = nat.fn(nat.hip_lib(), "qd_gather_cursor", [_p, _l, _p, _p, _p, _p, _p, _p, _l, _p, _p, _p, _l, _i, _i, _i,
                                                            _i, _i, _i, _p, _p])
            rp = self.rowpow if (hdce and self.rowpow is not None) else None
            xq = self.xq if classifier else None
            assert not classifier or xq is not None
            sc = self.den_scale if rp else None
            if sc is not None:   # (reads the cursor before the gather below advances it)
                fd = nat.fn(nat.hip_lib(), "qd_den_scale", [_p, _l, _p, _i, _i, _i, _p, _p, _l, _i, _p, _p])
                nat.check(fd(nat.ptr(perm), perm.numel(), nat.ptr(cursor), self.adv, self.off, self.B, nat.ptr(rp[0]),
                             nat.ptr(rp[1]) if rp[1] is not None else None, HL.stride(0) // cols, self.S, nat.ptr(sc),
                             nat.stream_ptr(Yp.device)), "den_scale")
            nat.check(f(nat.ptr(perm), perm.numel(), nat.ptr(cursor), nat.ptr(done) if done is not None else None,
                        nat.ptr(rp[0]) if rp else None, nat.ptr(rp[1]) if rp and rp[1] is not None else None,
                        nat.ptr(self.rowden) if rp else None, nat.ptr(Yp), Yp.stride(0),
                        nat.ptr(self.x1) if hdce else None, nat.ptr(xq) if xq is not None else None,
                        nat.ptr(self.rowoff) if hdce else None, HL.stride(0) // cols, self.E, self.U, self.B,
                        self.plane, self.off, self.adv, nat.ptr(sc) if sc is not None else None,
                        nat.stream_ptr(Yp.device)), "gather_cursor")
            return
        c = int(cursor.item())
        if c < 0 or c + self.adv > perm.numel():
            c = 0
        idx = perm[c + self.off:c + self.off + self.B]
        xq_saved = self.xq
        if not classifier:
            self.xq = None
        try:
            if hdce and self.den_global is not None:   # (strong scaling, torch NMSE: the global batch's powers)
                gl = perm[c:c + self.adv]
                self.den_global[:, 0] = HL.index_select(1, gl).pow(2).sum((1, 2))
                self.den_global[:, 1] = store.Hperf.index_select(1, gl).pow(2).sum((1, 2))
            if hdce:
                self(store, idx)
                if self.rowpow is not None:
                    o = self.rowoff.long()
                    self.rowden[:, 0] = self.rowpow[0][o]
                    self.rowden[:, 1] = self.rowpow[1][o] if self.rowpow[1] is not None else 0.0
                    if self.den_scale is not None:   # (strong scaling: see den_scale)
                        gl = perm[c:c + self.adv]
                        lsr = HL.stride(0) // cols
                        rows = (torch.arange(self.S, device=gl.device).view(-1, 1) * lsr + gl.view(1, -1))
                        sc = self._scales(rows, o, lsr)
                        self.den_scale.copy_(sc)
                        s_of_row = (o // lsr)
                        self.rowden.mul_(sc[s_of_row])
            elif classifier:
                g = Yp.index_select(1, idx)
                self.xq.copy_(g.reshape(self.S * self.B, 2, self.H, self.W))
        finally:
            self.xq = xq_saved
        if done is not None:
            cursor.fill_(c + self.adv)

    def _scales(self, rows: torch.Tensor, o: torch.Tensor, lsr: int) -> torch.Tensor:
        """(CPU strong scaling) per stream (global / part) label and perf powers (see den_scale)."""
        out = torch.ones(self.S, 2, device=rows.device)
        s_of_row = o // lsr
        for j, rp in enumerate(self.rowpow):
            if rp is None:
                continue
            g = rp[rows].sum(1)
            part = torch.zeros(self.S, device=rows.device, dtype=rp.dtype).index_add_(0, s_of_row, rp[o])
            out[:, j] = torch.where(part > 0, g / part.clamp_min(1e-30), torch.ones_like(g))
        return out

    def __call__(self, store, idx: torch.Tensor) -> None:
        Yp, HL = store.Yp, store.Hlabel
        S, N = Yp.shape[:2]
        assert S == self.S and idx.shape == (self.B,) and idx.dtype == torch.int64
        assert Yp.dtype == torch.float32 and Yp[0, 0].is_contiguous() and Yp.stride(1) == self.plane
        cols = HL.shape[-1]
        assert HL.stride(1) == cols and HL.stride(0) % cols == 0 and store.Hperf.stride() == HL.stride()
        if Yp.is_cuda:
            f = nat.fn(nat.hip_lib(), "qd_gather_step", [_p, _p, _l, _p, _p, _p, _l, _i, _i, _i, _i, _p])
            nat.check(f(nat.ptr(idx), nat.ptr(Yp), Yp.stride(0), nat.ptr(self.x1),
                        nat.ptr(self.xq) if self.xq is not None else None, nat.ptr(self.rowoff), HL.stride(0) // cols,
                        self.E, self.U, self.B, self.plane, nat.stream_ptr(Yp.device)), "gather_step")
            return
        E, U, B = self.E, self.U, self.B
        g = Yp.index_select(1, idx)                                   # (S, B, 2, H, W), s = e*U + u
        self.x1.copy_(g.view(E, U, B, 2, self.H, self.W).permute(1, 2, 0, 3, 4, 5)
                      .reshape(U * B, E * 2, self.H, self.W))
        if self.xq is not None:
            self.xq.copy_(g.reshape(self.S * B, 2, self.H, self.W))
        s = (torch.arange(E).view(1, 1, E) * U + torch.arange(U).view(U, 1, 1)).to(idx.device)
        off = s * (HL.stride(0) // cols) + idx.view(1, B, 1)
        self.rowoff.copy_(off.expand(U, B, E).reshape(-1).to(torch.int32))
