"""Classical scenario classifier SC_P128 on the HIP kernels (csrc/hip/sc.hip).

Reference: SC_P128 (Estimators_QuantumNAT_onchipQNN.py:79-101), trained with the mean NLL over the 9
streams (helpers Runner_P128_QuantumNAT_onchipQNN.py:285-302) and evaluated for the classical routing
of Test.py:158.  One training step over B samples is 4 launches, no autograd:
  sc_fwd     conv-ReLU-pool x2 + Linear + log_softmax + NLL (+ saved pool maps / argmax codes, dlogits)
  sc_finish  loss, correct count, NaN-guard flag (fixed-order sums)
  sc_bwd     every weight gradient as one slab row per workgroup (flat-parameter layout)
  slab sum   -> the FlatParamSpace gradient (overwrite or accumulate)
Inference (``forward`` / ``predict``) is the forward kernel alone.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch

from .. import _native as nat
from ..ops.optim import FlatParamSpace
from .slabsum import SlabBatch

_p, _i = ctypes.c_void_p, ctypes.c_int


class SCStepHIP:
    SPB_FWD = 4    # samples per forward workgroup
    SPB_BWD = 8    # samples per backward workgroup (one slab row each)

    def __init__(self, model, space: FlatParamSpace, batch_total: int = 0):
        self.m, self.space = model, space
        H, W = _grid(model)
        self.H, self.W = H, W
        names = dict(zip(space.names, space.offsets))
        o = [names["conv1.weight"], names["conv2.weight"], names["FC.weight"], names["FC.bias"]]
        F = model.flat
        # the kernel's slab row is the flat layout: the four tensors back to back (each a multiple of 16)
        assert o == [0, 576, 576 + 9216, 576 + 9216 + 3 * F] and space.numel == o[3] + 16, (o, space.numel)
        self.offs = (ctypes.c_int * 5)(*(o + [space.numel]))
        self.B = batch_total
        self.dev = space.flat.device
        self.out = torch.zeros(2, device=self.dev)          # (loss, correct)
        self.loss = self.out[0:1]
        self._bufs: Dict[int, tuple] = {}
        lib = nat.hip_lib()
        self._fwd = nat.fn(lib, "qd_sc_fwd", [_p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p])
        self._bwd = nat.fn(lib, "qd_sc_bwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p])
        self._fin = nat.fn(lib, "qd_sc_finish", [_p, _i, _i, _p, _p, _p, _i, _p])

    def _buf(self, B: int):
        b = self._bufs.get(B)
        if b is None:
            d, F, hw2 = self.dev, self.m.flat, 32 * (self.H // 2) * (self.W // 2)
            nf, nb = -(-B // self.SPB_FWD), -(-B // self.SPB_BWD)
            b = (torch.empty(B, hw2, device=d), torch.empty(B, hw2, device=d, dtype=torch.uint8),
                 torch.empty(B, F, device=d), torch.empty(B, F, device=d, dtype=torch.uint8),
                 torch.empty(B, 4, device=d), torch.empty(nf, 2, device=d),
                 torch.empty(nb, self.space.numel, device=d), nf, nb)
            self._bufs[B] = b
        return b

    def __call__(self, x: torch.Tensor, labels: torch.Tensor, loss_acc: Optional[torch.Tensor] = None,
                 skip: Optional[torch.Tensor] = None, skip_add: bool = False, accumulate: bool = True,
                 slabs: Optional[SlabBatch] = None) -> torch.Tensor:
        """x (B, 2, H, W) fp32 contiguous, labels (B,) int64: one training step's forward + backward; the
        gradients land in the flat space (``accumulate`` or overwrite).  Returns the mean NLL (1,)."""
        B = x.shape[0]
        assert x.is_contiguous() and x.dtype == torch.float32 and labels.dtype == torch.int64 and labels.numel() == B
        p1, c1, p2, c2, dl, part, slab, nf, nb = self._buf(B)
        st = nat.stream_ptr(x.device)
        flat = self.space.flat
        nat.check(self._fwd(nat.ptr(x), nat.ptr(flat), self.offs, nat.ptr(labels), B, self.SPB_FWD, self.H, self.W,
                            nat.ptr(p1), nat.ptr(c1), nat.ptr(p2), nat.ptr(c2), nat.ptr(dl), nat.ptr(part), None, None,
                            st), "sc_fwd")
        nat.check(self._fin(nat.ptr(part), nf, B, nat.ptr(self.out), nat.ptr(loss_acc) if loss_acc is not None else None,
                            nat.ptr(skip) if skip is not None else None, int(skip_add), st), "sc_finish")
        nat.check(self._bwd(nat.ptr(x), nat.ptr(flat), self.offs, B, self.SPB_BWD, self.H, self.W, nat.ptr(p1),
                            nat.ptr(c1), nat.ptr(p2), nat.ptr(c2), nat.ptr(dl), nat.ptr(slab), st), "sc_bwd")
        sb = slabs if slabs is not None else SlabBatch()
        sb.add(slab, self.space.grad, 1, nb, self.space.numel)
        if slabs is None:
            sb.launch(accumulate, st)
        return self.loss

    def forward(self, x: torch.Tensor, pred: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Inference: log-probabilities (B, 3) (and the argmax into ``pred`` (B,) int64 when given)."""
        B = x.shape[0]
        x = x.contiguous().float()
        logp = torch.empty(B, 3, device=x.device)
        nat.check(self._fwd(nat.ptr(x), nat.ptr(self.space.flat), self.offs, None, B, self.SPB_FWD, self.H, self.W,
                            None, None, None, None, None, None, nat.ptr(logp),
                            nat.ptr(pred) if pred is not None else None, nat.stream_ptr(x.device)), "sc_fwd")
        return logp

    def predict(self, x: torch.Tensor) -> torch.Tensor:
        pred = torch.empty(x.shape[0], device=x.device, dtype=torch.int64)
        self.forward(x, pred)
        return pred


def _grid(model):
    from ..models.estimators import pilot_grid
    return pilot_grid(model.pilot_num)
