"""Fused QSC training step on the HIP kernels (csrc/hip/qsc.hip + csrc/hip/qsim{,_big}.hip).

Reference step (Runner_P128_QuantumNAT_onchipQNN.py:341-369): 9 forward calls of
``QSC_P128`` (preprocess CNN -> PennyLane TorchLayer -> Linear -> log_softmax), summed
``nll_loss / 9``, one autograd backward, optional pruning, AdamW.

Here one step over all 9*B samples is 6 launches, no autograd:
  qsc_pre_fwd   CNN preprocess + Linear + tanh            -> angles (B, n)
  qsim_fwd      variational circuit                         -> E = <Z_i> (B, n)
  qsc_head      Linear(n, C) + log_softmax + mean NLL + backward -> loss, dE, dWc, dbc
  qsim_bwd      adjoint differentiation                     -> d angles, weight-grad slab
  reduce_slab   -> qlayer.weights grad
  qsc_pre_bwd   recompute + backprop the preprocess         -> slab -> flat grad (one column sum)
All gradients land in the model's FlatParamSpace; every buffer is static (graph-capturable).
QuantumNAT: each of the G streams gets its own noise draw w + sigma*N(0,1) (the reference
draws per forward call), generated in-kernel (qd_qnoise, one launch per step); forward AND
backward use it, the grads flow to the clean master.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from .. import _native as nat
from .slabsum import SlabBatch
from ..ops.optim import FlatParamSpace
from ..knobs import KNOBS
from ..ops.quantum import HIP_REG_MAX_QUBITS, stream_sim_ok

_p, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float


def balanced_grid(samples: int, waves: int, cap: int) -> int:
    """The fewest workgroups (<= cap) of ``waves`` one-sample-at-a-time waves that give every wave the same number
    of samples as a grid of ``cap`` gives its busiest wave: 192 for 2304 samples, 4 waves, cap 256."""
    spw = -(-samples // (waves * cap))
    return -(-samples // (waves * spw))


class QSCStepHIP:
    def __init__(self, model, space: FlatParamSpace, batch_total: int, n_groups: int = 1,
                 grid_fwd: int = 512, grid_bwd: int = 256, impl: str = "mfma", balance_bwd: bool = True):
        """impl: "mfma" (csrc/hip/qsc_mfma.hip: one wave per sample, fp32 MFMA convs; default) or
        "ref" (csrc/hip/qsc.hip: one workgroup per sample, VALU convs).  balance_bwd (mfma): shrink the
        backward's grid below ``grid_bwd`` until every wave takes the same number of samples."""
        self.m = model
        self.space = space
        dev = space.flat.device
        self.B = batch_total
        self.G = n_groups
        self.n = model.num_qubits
        self.L = model.n_layers
        self.C = model.n_classes
        pre = model.preprocess
        names = dict(zip(space.names, space.offsets))
        o = [names["preprocess.0.weight"], names["preprocess.0.bias"], names["preprocess.3.weight"],
             names["preprocess.3.bias"], names["preprocess.7.weight"], names["preprocess.7.bias"]]
        # slab row = flat columns [base, base + row): the preprocess grads (+ for the MFMA backward, which
        # also reduces the quantum layer's adjoint slab, the quantum weights in front of them)
        qoff = names["qlayer.weights"]
        base = min(o[0], qoff) if impl == "mfma" else o[0]
        row = o[5] + self.n - base
        row += (-row) % 4   # float4 slab sums; the tail lands in the flat space's alignment padding (zeros)
        assert base + row <= space.numel and (impl != "mfma" or qoff + 2 * self.n * self.L <= base + row)
        self.offs = (ctypes.c_int * 9)(*(o + [row, base, qoff]))
        self.row0, self.row = base, row
        feat = pre[7].weight.shape[1]
        self.Hh, self.Ww = (16, 8) if feat == 256 else (16, 16)
        self.impl = impl
        f32 = dict(device=dev, dtype=torch.float32)
        self.F = feat
        if impl == "mfma":
            wf = nat.fn(nat.hip_lib(), "qd_qsc2_waves", [_i, _i])
            self.grid_fwd = -(-batch_total // wf(self.Ww, 0))      # one sample per wave
            # at most 256 workgroups (grid-stride loop over the samples): the forward runs beside the HDCE
            # conv forward and leaves it more CUs -- 1 % per step over one sample per wave (576 workgroups
            # at 2304 samples) in 4 of 4 same-box rounds (profiles/r2_20_*)
            self.grid_fwd = min(self.grid_fwd, KNOBS.qsc_fwd_cap)
            self.grid_bwd = min(-(-batch_total // wf(self.Ww, 1)), grid_bwd)
            if balance_bwd:
                # the workgroup's slab reduction waits for its slowest wave: at 2304 samples 256 workgroups of
                # 4 waves give a quarter of the waves a third sample; 192 give every wave 3 (same box, 3 alternating
                # rounds: 0.3780-0.3792 against 0.3806-0.3825 ms, profiles/r6_06_qsc_grid_fp8_ab.txt)
                self.grid_bwd = balanced_grid(batch_total, wf(self.Ww, 1), self.grid_bwd)
            self.p2 = torch.empty(batch_total, feat, **f32)        # pool-2 features (linear weight grad)
            # saved by the forward for the backward: pool-1 map + both pools' argmax choices
            hw2 = self.Hh * self.Ww // 4
            self.p1s = torch.empty(batch_total, hw2 * 16, **f32)
            self.c1 = torch.empty(batch_total, hw2, device=dev, dtype=torch.int32)
            self.c2 = torch.empty(batch_total, feat, device=dev, dtype=torch.uint8)
            self.dpre = torch.empty(batch_total, self.n, **f32)
            self.gwl = space.grad[names["preprocess.7.weight"]:names["preprocess.7.weight"] + self.n * feat].view(
                self.n, feat)
            # the backward kernel also reduces dWl = dpre^T p2 into its slab when it fits; else a GEMM
            self.wl_in_kernel = bool(nat.fn(nat.hip_lib(), "qd_qsc2_wl_in_kernel", [_i, _i, _i])(
                self.Hh, self.Ww, self.n))
            if not self.wl_in_kernel:   # (the outer-product partials of qd_outer_partial: 36 samples per chunk)
                self.wl_bs = 36
                self.wlslab = torch.empty(-(-batch_total // self.wl_bs), self.n * feat, **f32)
        else:
            self.grid_fwd = min(grid_fwd, batch_total)
            self.grid_bwd = min(grid_bwd, batch_total)
        self.angles = torch.empty(batch_total, self.n, **f32)
        self.E = torch.empty(batch_total, self.n, **f32)
        self.dE = torch.empty(batch_total, self.n, **f32)
        self.dang = torch.empty(batch_total, self.n, **f32)
        self.loss = torch.zeros(1, **f32)
        self.preslab = torch.empty(self.grid_bwd, row, **f32)
        L = nat.hip_lib()
        self.big = self.n > HIP_REG_MAX_QUBITS  # workgroup-per-sample simulator (qsim_big.hip)
        # n = 12: every gate layer -- forward and adjoint -- as complex MFMA mode products (csrc/hip/qsim12_mfma.hip,
        # same contract as qsim_big.hip's kernels); knobs.KNOBS.qsim_mfma12 = False: the VALU kernels
        self.mfma12 = dev.type == "cuda" and self.n == 12 and 1 <= self.L <= 8 and KNOBS.qsim_mfma12
        # n = 13..16 with >= 2 layers: the streamed simulator (csrc/hip/qsim_stream.hip, one workgroup per
        # (sample, 4096-amplitude brick) per pass); else qsim_big.hip's workgroup-per-sample kernels
        self.stream = self.big and stream_sim_ok(self.n, self.L)
        if self.stream:
            self.qrows = nat.fn(L, "qd_qsim_stream_rows", [_i])(batch_total)
            ws = nat.fn(L, "qd_qsim_stream_workspace", [_i, _i, _i, _i], ctypes.c_longlong)
            nb = max(ws(self.n, batch_total, self.L, 0), ws(self.n, batch_total, self.L, 1))
            self.qws = torch.empty(nb, dtype=torch.uint8, device=dev)
            # the forward keeps every layer's pass-A output (L - 1 states: the backward's psi, never un-applied)
            sv = nat.fn(L, "qd_qsim_stream_save_bytes", [_i, _i, _i], ctypes.c_longlong)(self.n, batch_total, self.L)
            self.psave = torch.empty(sv, dtype=torch.uint8, device=dev)
        elif self.big:
            self.qrows = nat.fn(L, "qd_qsim_big_grid", [_i])(batch_total)
            if self.mfma12:
                # the per-(group, layer) MFMA operand images of the 12-qubit simulator (csrc/hip/qsim12_mfma.hip)
                nb = nat.fn(L, "qd_qsim_mfma12_workspace", [_i, _i], ctypes.c_longlong)(max(1, n_groups), self.L)
            else:
                ws = nat.fn(L, "qd_qsim_big_workspace", [_i, _i, _i], ctypes.c_longlong)
                nb = max(ws(self.n, self.qrows, 0), ws(self.n, self.qrows, 1))
            self.qws = torch.empty(nb, dtype=torch.uint8, device=dev) if nb else None
            # every sample's final state, kept by the forward for the adjoint backward (which then
            # skips re-running the circuit): 2304 x 2^16 x 8 B = 1.2 GB at 16 qubits -- HBM has room
            self.psave = torch.empty(batch_total * (8 << self.n), dtype=torch.uint8, device=dev)
        else:
            self.qrows = nat.fn(L, "qd_qsim_bwd_grid", [_i, _i])(self.n, batch_total)
            self.qws = None
        self.qslab = torch.empty(self.qrows, 2 * self.n * self.L, **f32)
        self._pre_fwd = nat.fn(L, "qd_qsc_pre_fwd", [_p, _p, _p, _p, _i, _i, _i, _i, _i, _p])
        self._pre_bwd = nat.fn(L, "qd_qsc_pre_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p])
        self._fwd2 = nat.fn(L, "qd_qsc2_fwd", [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p])
        self._bwd2 = nat.fn(L, "qd_qsc2_bwd", [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i,
                                                   _i, _p])
        # the preprocess CNN's products on bf16x3 MFMAs (fp32-grade: hi/lo bf16 operands, three products):
        # the forward's conv2 (qd_qsc2_fwd3) and, at P128, the whole backward (qsc2_bwd3_kernel); the f32
        # MFMA they replace runs at 1/16 of the bf16 rate.
        self._fwd3 = nat.fn(L, "qd_qsc2_fwd3", [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p, _p])
        self._bwd3 = nat.fn(L, "qd_qsc2_bwd3", [_p] * 12 + [_i] * 7 + [_p, _p])
        # (P256: KNOBS.qsc_fwd3_p256 -- the bf16x3 forward at 256 VGPRs halved its occupancy before round 6)
        self.fwd_x3 = (self.Hh, self.Ww) == (16, 8) or ((self.Hh, self.Ww) == (16, 16) and KNOBS.qsc_fwd3_p256)
        self.bwd_x3 = (self.Hh, self.Ww) == (16, 8)
        # the backward's bf16 hi / lo transposed conv2 weights, written by the bf16x3 forward each step
        self.w2t_img = torch.empty(2 * 9 * 16 * 48, device=self.p2.device, dtype=torch.bfloat16) \
            if (self.bwd_x3 and impl == "mfma") else None
        self._img_step = False   # the image holds this step's weights (the last forward was fwd3)
        self._head = nat.fn(L, "qd_qsc_head", [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p])
        if self.big:
            pre = "qd_qsim_stream" if self.stream else ("qd_qsim_mfma12" if self.mfma12 else "qd_qsim_big")
            self._qf = nat.fn(L, pre + "_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
            self._qb = nat.fn(L, pre + "_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
        else:
            # the forward keeps every sample's final state (2^n complex, 4.7 MB at 8 qubits) for the
            # adjoint backward, which then skips re-running the circuit
            self.psave = torch.empty(batch_total * (8 << self.n), dtype=torch.uint8, device=dev)
            self._qf = nat.fn(L, "qd_qsim_fwd_save", [_p, _p, _p, _i, _i, _i, _i, _p, _p])
            self._qb = nat.fn(L, "qd_qsim_bwd_saved", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p])
        self._rs = nat.fn(L, "qd_reduce_slab", [_p, _p, _i, _i, _f, _p])
        self._ssum = nat.fn(L, "qd_slab_rows_sum", [_p, _p, _i, _i, _i, _i, _p])
        self._outer = nat.fn(L, "qd_outer_partial", [_p, _p, _p, _i, _i, _i, _i, _p])
        self._qnoise = nat.fn(L, "qd_qnoise", [_p, _p, _i, _i, _f, ctypes.c_ulonglong, _p, _p])
        wq = model.qlayer.weights
        self.wnoisy = torch.empty((n_groups,) + tuple(wq.shape), **f32)
        self.noise_ctr = torch.zeros(1, dtype=torch.int64, device=dev)      # advanced by the kernel
        self.noise_seed = int(torch.randint(0, 2 ** 62, (1,)).item())       # from the (seeded) host RNG
        # n = 8: the circuit forward on the matrix cores (csrc/hip/qsim_mfma.hip: each layer's rotations as
        # Kronecker-factored complex products on mfma_f32_16x16x32_f16, fp16 hi/lo split = fp32-grade
        # amplitudes); its per-step operand images are built in the QuantumNAT noise draw's launch
        # (qd_qsim_mfma_prep_noise), so the step has no extra launch.  The adjoint backward reads the final
        # state it saves (qsim.hip's layout).  knobs.KNOBS.qsim_mfma = False: the register forward (qsim.hip).
        self.mfma = (dev.type == "cuda" and not self.big and self.n == 8 and 2 <= self.L <= 8
                     and self.psave is not None and KNOBS.qsim_mfma)
        if self.mfma:
            halves = nat.fn(L, "qd_qsim_mfma_ops_halves", [_i, _i], ctypes.c_longlong)(max(1, n_groups), self.L)
            self.qops = torch.empty(halves, dtype=torch.float16, device=dev)
            self.qdone = torch.zeros(1, dtype=torch.int32, device=dev)
            self._mprep = nat.fn(L, "qd_qsim_mfma_prep", [_p, _p, _i, _i, _p])
            self._mprep_noise = nat.fn(L, "qd_qsim_mfma_prep_noise",
                                       [_p, _p, _p, _i, _i, _f, ctypes.c_ulonglong, _p, _p, _p])
            self._mfwd = nat.fn(L, "qd_qsim_mfma_fwd", [_p, _p, _p, _p, _i, _i, _i, _p, _p])
        # n = 8: the adjoint backward on the matrix cores too (csrc/hip/qsim12_mfma.hip qd_qsim_mfma8_bwd: the same
        # contract as qd_qsim_bwd_saved, plus its own operand images); knobs.KNOBS.qsim_mfma_bwd = False: qsim.hip
        self.mfma_bwd = (dev.type == "cuda" and not self.big and self.n == 8 and 1 <= self.L <= 8
                         and self.psave is not None and KNOBS.qsim_mfma_bwd)
        if self.mfma_bwd:
            nb = nat.fn(L, "qd_qsim_mfma8_workspace", [_i, _i], ctypes.c_longlong)(max(1, n_groups), self.L)
            self.qops8 = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
            self._qb = nat.fn(L, "qd_qsim_mfma8_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])

    def quantum_weights(self) -> torch.Tensor:
        """Master weights, or (training + QuantumNAT) G per-stream noisy copies drawn in-kernel
        (qd_qnoise: counter-based RNG, one launch, no graph RNG state)."""
        m = self.m
        w = m.qlayer.weights.detach()
        if m.training and m.use_quantumnat and m.noise_level > 0:
            if self.mfma:   # the draw + the MFMA forward's operand images of the noisy layers, one launch
                nat.check(self._mprep_noise(nat.ptr(w), nat.ptr(self.wnoisy), nat.ptr(self.qops), self.G, self.L,
                                            float(m.noise_level), self.noise_seed, nat.ptr(self.noise_ctr),
                                            nat.ptr(self.qdone), nat.stream_ptr(w.device)), "qsim_mfma_prep_noise")
            else:
                nat.check(self._qnoise(nat.ptr(w), nat.ptr(self.wnoisy), self.G, w.numel(), float(m.noise_level),
                                       self.noise_seed, nat.ptr(self.noise_ctr), nat.stream_ptr(w.device)), "qnoise")
            return self.wnoisy
        if self.mfma:
            w = w.contiguous()
            nat.check(self._mprep(nat.ptr(w), nat.ptr(self.qops), 1, self.L, nat.stream_ptr(w.device)), "qsim_mfma_prep")
        return w

    @torch.no_grad()
    def _fwd_mfma(self, x, flat, st) -> None:
        """The preprocess forward (f32 or bf16x3 conv2); the bf16x3 one also refreshes the backward's W2T image."""
        args = (nat.ptr(x), nat.ptr(flat), self.offs, nat.ptr(self.angles), nat.ptr(self.p2), *self._saved(), self.B,
                self.n, self.Hh, self.Ww, self.grid_fwd)
        if self.fwd_x3:
            img = self.w2t_img if self.bwd_x3 else None
            nat.check(self._fwd3(*args, nat.ptr(img) if img is not None else None, st), "qsc2_fwd3")
            self._img_step = img is not None
        else:
            nat.check(self._fwd2(*args, st), "qsc2_fwd")
            self._img_step = False

    def _saved(self):
        return nat.ptr(self.p1s), nat.ptr(self.c1), nat.ptr(self.c2)

    def __call__(self, x: torch.Tensor, labels: torch.Tensor, loss_acc: Optional[torch.Tensor] = None,
                 skip: Optional[torch.Tensor] = None, skip_add: bool = False, accumulate: bool = True,
                 slabs: Optional[SlabBatch] = None) -> torch.Tensor:
        """x (B, 2, H, W) fp32 contiguous, labels (B,) int64.  Returns loss (1,).
        ``skip`` (fp32 (1,)): set (or, with skip_add, incremented) to 1 if the loss is not finite.
        ``accumulate``: add into the grads (default) or write them (every grad of the model has exactly
        one producer per step, so a zero_grad before the step becomes unnecessary).
        ``slabs``: queue the gradient-slab reductions on this batch (the caller launches it with the
        same ``accumulate``) instead of launching them here."""
        self.forward_part(x, labels, loss_acc, skip, skip_add, accumulate)
        return self.backward_part(x, accumulate, slabs)

    def forward_part(self, x: torch.Tensor, labels: torch.Tensor, loss_acc: Optional[torch.Tensor] = None,
                     skip: Optional[torch.Tensor] = None, skip_add: bool = False, accumulate: bool = True) -> None:
        """First half of ``__call__``: preprocess, noise draw, simulator forward, head (loss, dE and
        the head's grads).  ``backward_part`` (same x) finishes the step -- the two halves can sit in
        different graphs of an execution plan."""
        m, sp = self.m, self.space
        B, n, L = self.B, self.n, self.L
        assert x.shape[0] == B and x.is_contiguous() and labels.dtype == torch.int64
        st = nat.stream_ptr(x.device)
        flat = sp.flat
        if self.impl == "mfma":
            self._fwd_mfma(x, flat, st)
        else:
            nat.check(self._pre_fwd(nat.ptr(x), nat.ptr(flat), self.offs, nat.ptr(self.angles), B, n, self.Hh,
                                    self.Ww, self.grid_fwd, st), "qsc_pre_fwd")
        w = self.quantum_weights().contiguous()
        wgroup = B // w.shape[0] if w.dim() == 4 else 0
        if wgroup and wgroup * w.shape[0] != B:   # (the kernels map sample s to group s // wgroup: G must divide B)
            raise ValueError(f"{w.shape[0]} QuantumNAT weight groups do not divide the batch of {B}")
        extra = (nat.ptr(self.qws) if self.qws is not None else None,
                 nat.ptr(self.psave) if self.psave is not None else None) if self.big else \
            (nat.ptr(self.psave) if self.psave is not None else None,)
        if self.mfma:
            nat.check(self._mfwd(nat.ptr(self.angles), nat.ptr(w), nat.ptr(self.qops), nat.ptr(self.E), B, L, wgroup,
                                 nat.ptr(self.psave), st), "qsim_mfma_fwd")
        else:
            nat.check(self._qf(nat.ptr(self.angles), nat.ptr(w), nat.ptr(self.E), B, n, L, wgroup, *extra, st),
                      "qsim_fwd")
        cls = m.classifier
        nat.check(self._head(nat.ptr(self.E), nat.ptr(cls.weight), nat.ptr(cls.bias), nat.ptr(labels),
                             nat.ptr(self.dE), nat.ptr(cls.weight.grad), nat.ptr(cls.bias.grad), nat.ptr(self.loss),
                             nat.ptr(loss_acc) if loss_acc is not None else None,
                             nat.ptr(skip) if skip is not None else None, int(skip_add), int(accumulate), B, n, self.C,
                             st), "qsc_head")
        self._w_cur = w

    @torch.no_grad()
    def infer(self, x: torch.Tensor, pred: Optional[torch.Tensor] = None,
              logp: Optional[torch.Tensor] = None) -> None:
        """Inference on the HIP kernels (x.shape[0] == B): preprocess CNN, the circuit with the clean
        master weights (no QuantumNAT noise), then a thread-per-sample head -> log-probabilities (B, C)
        and / or the argmax (B,) int64."""
        m = self.m
        B, n, L = self.B, self.n, self.L
        assert x.shape[0] == B and x.is_contiguous() and self.impl == "mfma"
        st = nat.stream_ptr(x.device)
        self._fwd_mfma(x, self.space.flat, st)
        w = m.qlayer.weights.detach().contiguous()
        extra = (nat.ptr(self.qws) if self.qws is not None else None,
                 nat.ptr(self.psave) if self.psave is not None else None) if self.big else \
            (nat.ptr(self.psave) if self.psave is not None else None,)
        nat.check(self._qf(nat.ptr(self.angles), nat.ptr(w), nat.ptr(self.E), B, n, L, 0, *extra, st), "qsim_fwd")
        cls = m.classifier
        f = nat.fn(nat.hip_lib(), "qd_qsc_infer_head", [_p, _p, _p, _p, _p, _i, _i, _i, _p])
        nat.check(f(nat.ptr(self.E), nat.ptr(cls.weight), nat.ptr(cls.bias), nat.ptr(logp) if logp is not None else None,
                    nat.ptr(pred) if pred is not None else None, B, n, self.C, st), "qsc_infer_head")

    def backward_part(self, x: torch.Tensor, accumulate: bool = True, slabs: Optional[SlabBatch] = None) -> torch.Tensor:
        m, sp = self.m, self.space
        B, n, L = self.B, self.n, self.L
        st = nat.stream_ptr(x.device)
        flat = sp.flat
        w = self._w_cur
        wgroup = B // w.shape[0] if w.dim() == 4 else 0
        if wgroup and wgroup * w.shape[0] != B:   # (the kernels map sample s to group s // wgroup: G must divide B)
            raise ValueError(f"{w.shape[0]} QuantumNAT weight groups do not divide the batch of {B}")
        extra = (nat.ptr(self.qws) if self.qws is not None else None,
                 nat.ptr(self.psave) if self.psave is not None else None) if self.big else \
            (nat.ptr(self.psave) if self.psave is not None else None,)
        if self.mfma_bwd:
            extra = (nat.ptr(self.qops8), nat.ptr(self.psave))
        nat.check(self._qb(nat.ptr(self.angles), nat.ptr(w), nat.ptr(self.dE), nat.ptr(self.dang),
                           nat.ptr(self.qslab), B, n, L, wgroup, *extra, st), "qsim_bwd")
        own = SlabBatch()
        if self.impl != "mfma":   # (the MFMA preprocess backward folds this reduction into its own slab)
            (slabs if slabs is not None else own).add(self.qslab, m.qlayer.weights.grad, 1, self.qrows, 2 * n * L)
        if self.impl == "mfma":
            args = (nat.ptr(x), nat.ptr(flat), self.offs, nat.ptr(self.angles), nat.ptr(self.dang), nat.ptr(self.dpre),
                    nat.ptr(self.preslab), nat.ptr(self.p2), *self._saved(), nat.ptr(self.qslab), self.qrows, 2 * n * L,
                    B, n, self.Hh, self.Ww, self.grid_bwd)
            if self.bwd_x3:
                nat.check(self._bwd3(*args, nat.ptr(self.w2t_img) if self._img_step else None, st), "qsc2_bwd3")
            else:
                nat.check(self._bwd2(*args, st), "qsc2_bwd")
        else:
            nat.check(self._pre_bwd(nat.ptr(x), nat.ptr(flat), self.offs, nat.ptr(self.dang), nat.ptr(self.preslab), B,
                                    n, self.Hh, self.Ww, self.grid_bwd, st), "qsc_pre_bwd")
        # (the linear-weight GEMM below overwrites columns of this slab's output: keep it in order)
        gemm_wl = self.impl == "mfma" and not self.wl_in_kernel
        (slabs if slabs is not None and not gemm_wl else own).add(self.preslab, sp.grad[self.row0:], 1,
                                                                   self.grid_bwd, self.row)
        own.launch(accumulate, st)
        if gemm_wl:
            # linear weight grad over the batch, dWl = dpre^T p2 (the slab row left these columns 0): per-chunk
            # outer-product partials + one slab reduction over the chunks (csrc/hip/qsc.hip qd_outer_partial)
            Bt, F = self.p2.shape
            nat.check(self._outer(nat.ptr(self.dpre), nat.ptr(self.p2), nat.ptr(self.wlslab), Bt, self.n, F,
                                  self.wl_bs, st), "qsc_outer_partial")
            nat.check(self._ssum(nat.ptr(self.wlslab), nat.ptr(self.gwl), 1, self.wlslab.shape[0], self.n * F,
                                 int(accumulate), st), "qsc_wl_slab_sum")
        return self.loss
