"""Test-time hierarchical estimation on the HIP kernels (the model side of ``Test.py``'s sweep).

Reference (Test.py:140-214): per test batch, classify the scenario with the classical SC and the quantum
SC, bucket the samples by predicted scenario in a Python loop, run each bucket through its expert
``Conv_s`` and the shared ``CE`` (all under DataParallel, on cuDNN / cuBLAS).

Here, per chunk of ``chunk`` samples (one static buffer set; graph-friendly, no host sync inside):
  gather      the chunk's pilots into the experts-in-channels conv input (csrc/hip/gather.hip with a
              zero stream stride: every expert's channel pair carries the same sample)
  classify    SC_P128: csrc/hip/sc.hip forward (argmax written in-kernel); QSC_P128: preprocess +
              circuit (clean master weights) + a thread-per-sample head (csrc/hip/qsc*.hip, qsim*.hip)
  experts     the conv / BN (running statistics) / ReLU stack of ALL experts on every sample
              (csrc/hip/conv.hip, one launch per layer): at these sizes evaluating the three small
              experts densely costs less than sorting samples into buckets
  routed FC   csrc/hip/gemm.hip forward GEMM whose A-operand loads read row ``i * E + expert[i]`` of the
              expert features: the top-1 routing is fused into the GEMM (no permutation, no scatter)
"""
from __future__ import annotations

import copy
import ctypes
from typing import Optional, Sequence

import torch
import torch.nn as nn

from .. import _native as nat
from ..models.estimators import QSC_P128, SC_P128, pilot_grid
from ..ops.optim import FlatParamSpace

_p, _i, _l = ctypes.c_void_p, ctypes.c_int, ctypes.c_long


class HIPInference:
    def __init__(self, convs: Sequence[nn.Module], fc: nn.Module, pilot_num: int, device, chunk: int = 2304,
                 sc: Optional[SC_P128] = None, qsc: Optional[QSC_P128] = None):
        from ..ops.conv import ConvStackHIP
        from ..ops.qsc import QSCStepHIP
        from ..ops.sc import SCStepHIP
        from .engine import HDCEModel
        self.dev = torch.device(device)
        self.chunk = chunk
        self.H, self.W = pilot_grid(pilot_num)
        self.E = len(convs)
        self.pilot_num = pilot_num
        # the estimator: an HDCEModel holding the checkpoint's experts + FC (its grouped buffers are what
        # the conv kernels read), eval mode
        m = HDCEModel(pilot_num, self.dev, "bf16", self.E)
        with torch.no_grad():
            for e in range(self.E):
                m.convs[e].load_state_dict(convs[e].state_dict())
            m.fc.load_state_dict(fc.state_dict())
        self.model = m
        self.conv = ConvStackHIP(m, 1, chunk)
        self.W_lp = m.fc_w.detach().to(torch.bfloat16).contiguous()
        self.b_lp = m.fc_b.detach().to(torch.bfloat16).contiguous()
        # classifiers: private copies whose parameters live in flat spaces (the kernels' layout)
        self.sc = self.qsc = None
        if sc is not None:
            self._sc_mod = copy.deepcopy(sc).to(self.dev).eval()
            self.sc = SCStepHIP(self._sc_mod, FlatParamSpace(list(self._sc_mod.named_parameters()), self.dev))
        if qsc is not None:
            self._qsc_mod = copy.deepcopy(qsc).to(self.dev).eval()
            self.qsc = QSCStepHIP(self._qsc_mod, FlatParamSpace(list(self._qsc_mod.named_parameters()), self.dev),
                                  chunk, n_groups=1)
        plane = 2 * self.H * self.W
        self.xq = torch.zeros(chunk, 2, self.H, self.W, device=self.dev)
        self.x1 = torch.zeros(chunk, 2 * self.E, self.H, self.W, device=self.dev)
        self.idx = torch.zeros(chunk, dtype=torch.int64, device=self.dev)
        self.pred = torch.zeros(chunk, dtype=torch.int64, device=self.dev)
        self.Y = torch.empty(chunk, self.W_lp.shape[0], device=self.dev, dtype=torch.bfloat16)
        self._gather = nat.fn(nat.hip_lib(), "qd_gather_step", [_p, _p, _l, _p, _p, _p, _l, _i, _i, _i, _i, _p])
        self._plane = plane

    @torch.no_grad()
    def refresh(self, convs: Sequence[nn.Module], fc: nn.Module) -> None:
        """Reload the estimator weights and BN statistics (e.g. once per epoch of a training run: the
        engine's buffers and static launch shapes are kept, the conv weights are re-packed by every forward)."""
        for e in range(self.E):
            self.model.convs[e].load_state_dict(convs[e].state_dict())
        self.model.fc.load_state_dict(fc.state_dict())
        self.W_lp.copy_(self.model.fc_w.detach())
        self.b_lp.copy_(self.model.fc_b.detach())

    @torch.no_grad()
    def load_bn_stats(self, convs: Sequence[nn.Module]) -> None:
        """Refresh the experts' BN running statistics (views into the grouped buffers the conv kernels
        read) from ``convs``, e.g. after a test-time BN re-estimation."""
        for e in range(self.E):
            src = [m for m in convs[e].modules() if isinstance(m, nn.BatchNorm2d)]
            dst = [m for m in self.model.convs[e].modules() if isinstance(m, nn.BatchNorm2d)]
            for d, s_ in zip(dst, src):
                d.running_mean.copy_(s_.running_mean)
                d.running_var.copy_(s_.running_var)

    @torch.no_grad()
    def recalibrate_bn(self, convs: Sequence[nn.Module], x: torch.Tensor, expert: torch.Tensor,
                       chunk: int = 4096) -> list:
        """Test-time BN re-estimation (``evaluate.recalibrate_bn``, the sweep's bn_adapt option) on the HIP
        training conv forward instead of MIOpen: every expert's BN running statistics become the cumulative
        average of its per-chunk batch statistics over the samples routed to it (torch's momentum=None rule,
        reproduced exactly as momentum 1/k for the k-th chunk of the kernels' running-stat update; chunks
        of fewer than 2 samples are skipped, as there).  Runs on a scratch copy of the experts (the other
        experts' channels of a launch get the same samples and are discarded), writes the new statistics
        into ``convs`` and returns their previous ones for ``evaluate.restore_bn``."""
        from ..ops.conv import ConvStackHIP
        from .engine import HDCEModel
        if getattr(self, "_rc_model", None) is None:
            self._rc_model = HDCEModel(self.pilot_num, self.dev, "bf16", self.E)
        m = self._rc_model
        stacks = {}
        x = x.to(self.dev).contiguous().float()
        expert = expert.to(self.dev)
        saved = []
        for e, conv in enumerate(convs):
            bns = [b for b in conv.modules() if isinstance(b, nn.BatchNorm2d)]
            saved.append([(b.momentum, b.running_mean.clone(), b.running_var.clone(), b.num_batches_tracked.clone())
                          for b in bns])
            xe = x[expert == e]
            n = xe.shape[0]
            if n < 2:
                continue
            m.convs[e].load_state_dict(conv.state_dict())
            dst = [b for b in m.convs[e].modules() if isinstance(b, nn.BatchNorm2d)]
            for d in dst:
                d.running_mean.zero_()
                d.running_var.fill_(1.0)
            k = 0
            for lo in range(0, n, chunk):
                c = min(chunk, n - lo)
                if c < 2:
                    continue
                k += 1
                if c not in stacks:
                    stacks[c] = (ConvStackHIP(m, 1, c),
                                 torch.empty(c, 2 * self.E, self.H, self.W, device=self.dev))
                stk, x1 = stacks[c]
                x1.view(c, self.E, 2, self.H, self.W).copy_(xe[lo:lo + c].view(c, 1, 2, self.H, self.W)
                                                            .expand(c, self.E, 2, self.H, self.W))
                m.momentum = 1.0 / k
                stk.forward(x1, training=True)
            m.momentum = 0.1
            for b, d in zip(bns, dst):
                b.running_mean.copy_(d.running_mean)
                b.running_var.copy_(d.running_var)
                b.num_batches_tracked.fill_(k)
        return saved

    def _load(self, x: torch.Tensor, lo: int, n: int) -> None:
        """Samples x[lo:lo+n] -> the classifier input (xq) and the experts-in-channels conv input (x1); the
        chunk's tail (n < chunk) repeats sample lo (its outputs are dropped)."""
        torch.arange(lo, lo + self.chunk, out=self.idx)
        self.idx.clamp_(max=lo + n - 1)
        st = nat.stream_ptr(self.dev)
        nat.check(self._gather(nat.ptr(self.idx), nat.ptr(x), 0, nat.ptr(self.x1), None, None, 0, self.E, 1,
                               self.chunk, self._plane, st), "gather(x1)")
        nat.check(self._gather(nat.ptr(self.idx), nat.ptr(x), 0, None, nat.ptr(self.xq), None, 0, 1, 1,
                               self.chunk, self._plane, st), "gather(xq)")

    @torch.no_grad()
    def classify(self, x: torch.Tensor, which: str) -> torch.Tensor:
        """Predicted scenario (N,) int64 of every sample with the classical ("classical") or quantum SC."""
        clf = self.sc if which == "classical" else self.qsc
        assert clf is not None, f"no {which} classifier loaded"
        x = x.contiguous().float()
        N = x.shape[0]
        out = torch.empty(N, dtype=torch.int64, device=self.dev)
        for lo in range(0, N, self.chunk):
            n = min(self.chunk, N - lo)
            self._load(x, lo, n)
            if which == "classical":
                self.sc.forward(self.xq, self.pred)
            else:
                self.qsc.infer(self.xq, self.pred)
            out[lo:lo + n].copy_(self.pred[:n])
        return out

    @torch.no_grad()
    def estimate(self, x: torch.Tensor, expert: torch.Tensor) -> torch.Tensor:
        """Routed estimate (N, 2048) fp32: sample i through expert ``expert[i]`` and the shared FC."""
        from ..ops.fc import gemm_fwd
        x = x.contiguous().float()
        N = x.shape[0]
        expert = expert.to(self.dev, torch.int64)
        out = torch.empty(N, self.W_lp.shape[0], device=self.dev)
        for lo in range(0, N, self.chunk):
            n = min(self.chunk, N - lo)
            self._load(x, lo, n)
            self.pred[:n].copy_(expert[lo:lo + n])
            h = self.conv.forward(self.x1, training=False)            # (chunk * E, 32 H W) bf16, rows (b, e)
            gemm_fwd(h, self.W_lp, self.b_lp, out=self.Y, expert=self.pred, n_experts=self.E)
            out[lo:lo + n].copy_(self.Y[:n])
        return out
