"""Per-stream NMSE loss with a fused gradient (csrc/hip/nmse.hip).

Reference: ``NMSE_cuda`` (Estimators_QuantumNAT_onchipQNN.py:282-286) applied per
stream and averaged over the 9 streams (Runner_P128_QuantumNAT_onchipQNN.py:194-199).

``StreamNMSE`` evaluates, for an activation Y whose rows belong to S streams,
  loss      = (1/S) sum_s sum_{r in s} |Y_r - L_r|^2 / sum_{r in s} |L_r|^2
  loss_perf = same against the perfect channel (monitor, R:113)
and returns dY = dloss/dY without autograd (the HDCE engine feeds it straight into
the FC backward).  The row->stream map is a device int32 tensor, so any row order
(e.g. the expert-interleaved order of the grouped estimator) works.

Labels can be read in place from the dataset store: set ``rowoff`` (int32, one store row per
output row, produced by ops/gather.py) and pass the (S, N, cols) label/perf stores instead of
(rows, cols) tensors -- the kernels index through it, so no permuted label copy is ever made.

In data-parallel runs ``sums()`` + all-reduce + ``finalize()`` give the GLOBAL NMSE
(sum of errors over sum of powers across ranks), never a mean of per-rank ratios.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from .. import _native as nat
from ..knobs import KNOBS

_p, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float


class LossFinish(ctypes.Structure):
    """csrc/hip/common.h LossFinish: the HDCE loss finish a later launch can host."""
    _fields_ = [("part", ctypes.c_void_p), ("dens", ctypes.c_void_p), ("ss", ctypes.c_void_p),
                ("loss", ctypes.c_void_p), ("skip", ctypes.c_void_p), ("gx", ctypes.c_int),
                ("chunks_per_u", ctypes.c_int), ("U", ctypes.c_int), ("E", ctypes.c_int)]


class StreamNMSE:
    def __init__(self, row_stream: torch.Tensor, n_streams: int, cols: int = 2048):
        self.row_stream = row_stream.to(torch.int32).contiguous()
        self.rows = row_stream.numel()
        self.S = n_streams
        self.cols = cols
        dev = row_stream.device
        self.rowsums = torch.zeros(self.rows, 4, device=dev)
        self.ss = torch.zeros(n_streams, 4, device=dev)       # (err, pow, err_perf, pow_perf) per stream
        self.loss = torch.zeros(2, device=dev)               # (loss, loss_perf)
        self.coef = torch.zeros(n_streams, device=dev)
        self.skip = torch.zeros(1, device=dev, dtype=torch.float32)  # NaN guard flag (all-reduced in DP)
        self._rs_long = self.row_stream.long()
        # fused path: rows per block = E * rpc_mult (scripts/probes/probe_nmse.py: 22.7 vs 24.2 us isolated at 4 vs 2;
        # 0.7 % per step in 2 of 2 rounds, profiles/r2_20_variants.md)
        self.rpc_mult = 4
        self.rowoff: Optional[torch.Tensor] = None
        # (S, 2) per-stream (label, perf) denominators of the GLOBAL batch, when this rank computes only part
        # of it (data parallelism with the reference's DataParallel semantics): the loss becomes this
        # rank's share sum_s num_s / den_global_s / S and the gradient coefficients 2 / (S den_global_s).
        # CPU path: used by finalize; GPU one-pass path: the caller scales its per-row powers instead.
        self.den_global: Optional[torch.Tensor] = None
        # CSR list of each stream's rows (stable order) for the one-launch reduce + finalize
        self.order = torch.sort(self._rs_long, stable=True).indices.to(torch.int32)
        cnt = torch.bincount(self._rs_long, minlength=n_streams)
        self.off = torch.cat([cnt.new_zeros(1), cnt.cumsum(0)]).to(torch.int32)

    def _labels(self, t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """Host-path view of the labels in output-row order."""
        if t is None or self.rowoff is None:
            return t
        # (S, N, cols) store, possibly a rank-shard view: rowoff = s * (stride0 / cols) + n
        sr = t.stride(0) // self.cols
        o = self.rowoff.long()
        return t[o // sr, o % sr]

    def _check_labels(self, t: torch.Tensor) -> None:
        assert t.dtype == torch.float32 and t.shape[-1] == self.cols and t.stride(-1) == 1
        if self.rowoff is None:
            assert t.shape == (self.rows, self.cols) and t.is_contiguous()

    def _row_sums_hip(self, Y, label, perf, st) -> None:
        self._check_labels(label)
        if perf is not None:
            self._check_labels(perf)
        f = nat.fn(nat.hip_lib(), "qd_nmse_row_sums", [_p, _i, _p, _p, _p, _p, _i, _i, _p])
        nat.check(f(nat.ptr(Y), int(Y.dtype == torch.bfloat16), nat.ptr(label),
                    nat.ptr(perf) if perf is not None else None,
                    nat.ptr(self.rowoff) if self.rowoff is not None else None, nat.ptr(self.rowsums), self.rows,
                    self.cols, st), "nmse_row_sums")

    def sums(self, Y: torch.Tensor, label: torch.Tensor, perf: Optional[torch.Tensor]) -> torch.Tensor:
        assert Y.shape == (self.rows, self.cols)
        if Y.is_cuda:
            lib = nat.hip_lib()
            st = nat.stream_ptr(Y.device)
            self._row_sums_hip(Y, label, perf, st)
            g = nat.fn(lib, "qd_nmse_stream_sums", [_p, _p, _p, _i, _i, _p])
            nat.check(g(nat.ptr(self.rowsums), nat.ptr(self.row_stream), nat.ptr(self.ss), self.rows, self.S, st),
                      "nmse_stream_sums")
        else:
            label, perf = self._labels(label), self._labels(perf)
            Yf = Y.float()
            rs = torch.stack([((Yf - label) ** 2).sum(1), (label ** 2).sum(1),
                              ((Yf - perf) ** 2).sum(1) if perf is not None else torch.zeros(self.rows),
                              (perf ** 2).sum(1) if perf is not None else torch.zeros(self.rows)], 1)
            self.ss.zero_().index_add_(0, self._rs_long, rs)
        return self.ss

    def sums_finalize(self, Y: torch.Tensor, label: torch.Tensor, perf: Optional[torch.Tensor],
                      loss_scale: float = 1.0) -> torch.Tensor:
        """sums() + finalize() for a rank-local loss; on the GPU the stream reduction and the
        finalisation are one launch."""
        if not Y.is_cuda:
            self.sums(Y, label, perf)
            return self.finalize(loss_scale)
        assert Y.shape == (self.rows, self.cols)
        lib = nat.hip_lib()
        st = nat.stream_ptr(Y.device)
        self._row_sums_hip(Y, label, perf, st)
        g = nat.fn(lib, "qd_nmse_reduce_finalize", [_p, _p, _p, _p, _p, _p, _p, _i, _f, _p])
        nat.check(g(nat.ptr(self.rowsums), nat.ptr(self.order), nat.ptr(self.off), nat.ptr(self.ss), nat.ptr(self.loss),
                    nat.ptr(self.coef), nat.ptr(self.skip), self.S, loss_scale, st), "nmse_reduce_finalize")
        return self.loss

    def finalize(self, loss_scale: float = 1.0) -> torch.Tensor:
        if self.ss.is_cuda:
            lib = nat.hip_lib()
            f = nat.fn(lib, "qd_nmse_finalize", [_p, _p, _p, _p, _i, _f, _p])
            nat.check(f(nat.ptr(self.ss), nat.ptr(self.loss), nat.ptr(self.coef), nat.ptr(self.skip), self.S,
                        loss_scale, nat.stream_ptr(self.ss.device)), "nmse_finalize")
        else:
            ss = self.ss
            den, denp = (ss[:, 1], ss[:, 3]) if self.den_global is None else (self.den_global[:, 0], self.den_global[:, 1])
            self.loss[0] = (ss[:, 0] / den).sum() / self.S
            self.loss[1] = (ss[:, 2] / denp.clamp_min(1e-30)).sum() / self.S
            self.coef.copy_(loss_scale * 2.0 / (self.S * den))
            self.skip.fill_(0.0 if torch.isfinite(self.loss[0]) else 1.0)
        return self.loss

    def grad(self, Y: torch.Tensor, label: torch.Tensor, out_dtype=torch.float32,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
        dY = out if out is not None else torch.empty(self.rows, self.cols, device=Y.device, dtype=out_dtype)
        if Y.is_cuda:
            lib = nat.hip_lib()
            self._check_labels(label)
            f = nat.fn(lib, "qd_nmse_grad", [_p, _i, _p, _p, _p, _p, _p, _i, _i, _i, _p])
            nat.check(f(nat.ptr(Y), int(Y.dtype == torch.bfloat16), nat.ptr(label), nat.ptr(self.coef),
                        nat.ptr(self.row_stream), nat.ptr(self.rowoff) if self.rowoff is not None else None,
                        nat.ptr(dY), int(dY.dtype == torch.bfloat16), self.rows, self.cols,
                        nat.stream_ptr(Y.device)), "nmse_grad")
        else:
            dY.copy_(self.coef[self._rs_long][:, None] * (Y.float() - self._labels(label)))
        return dY

    def grad_bias(self, Y: torch.Tensor, label: torch.Tensor, bias_grad: torch.Tensor, out_dtype=torch.float32,
                  chunks: int = 128) -> torch.Tensor:
        """dY (as ``grad``) and, fused into the same pass, the FC bias gradient sum_rows dY written
        (overwritten) into ``bias_grad``: per-row-chunk column sums + one deterministic slab reduce."""
        dY = torch.empty(self.rows, self.cols, device=Y.device, dtype=out_dtype)
        if not Y.is_cuda:
            dY.copy_(self.coef[self._rs_long][:, None] * (Y.float() - self._labels(label)))
            bias_grad.copy_(dY.float().sum(0))
            return dY
        if getattr(self, "_colsum", None) is None or self._colsum.shape[0] != chunks:
            self._colsum = torch.empty(chunks, self.cols, device=Y.device)
        lib = nat.hip_lib()
        self._check_labels(label)
        f = nat.fn(lib, "qd_nmse_grad_bias", [_p, _i, _p, _p, _p, _p, _p, _i, _p, _i, _i, _i, _p])
        st = nat.stream_ptr(Y.device)
        nat.check(f(nat.ptr(Y), int(Y.dtype == torch.bfloat16), nat.ptr(label), nat.ptr(self.coef),
                    nat.ptr(self.row_stream), nat.ptr(self.rowoff) if self.rowoff is not None else None,
                    nat.ptr(dY), int(dY.dtype == torch.bfloat16), nat.ptr(self._colsum), chunks, self.rows,
                    self.cols, st), "nmse_grad_bias")
        ssum = nat.fn(lib, "qd_slab_rows_sum", [_p, _p, _i, _i, _i, _i, _p])
        nat.check(ssum(nat.ptr(self._colsum), nat.ptr(bias_grad), 1, chunks, self.cols, 0, st), "bias_grad_sum")
        return dY

    # ------------------------------------------------------------------ one-pass GPU path
    def _row_powers(self, t: torch.Tensor) -> torch.Tensor:
        """sum |row|^2 of every row of a (S, N, cols) store view, laid out in rowoff's row space
        (s * stride0/cols + n) -- dataset constants, computed once per store."""
        key = (t.data_ptr(), tuple(t.shape), tuple(t.stride()))
        cache = self.__dict__.setdefault("_rowpow", {})
        if key not in cache:
            S, N, cols = t.shape
            sr = t.stride(0) // cols
            out = torch.zeros(S * sr, device=t.device, dtype=torch.float32)
            out.view(S, sr)[:, :N] = t.float().pow(2).sum(-1)
            cache[key] = out
        return cache[key]

    def fused(self, Y: torch.Tensor, label: torch.Tensor, perf: Optional[torch.Tensor], bias_grad: torch.Tensor,
              layout: Tuple[int, int, int], out_dtype=torch.bfloat16, loss_scale: float = 1.0,
              rpc_mult: Optional[int] = None, rowden: Optional[torch.Tensor] = None,
              bias_slabs=None, defer_loss: bool = False) -> torch.Tensor:
        """GPU, labels through ``rowoff``, rows in (u, b, e) order with ``layout`` = (E, U, B): loss,
        loss_perf, skip, dY and the bias gradient (overwritten into ``bias_grad``) in TWO launches
        (csrc/hip/nmse.hip qd_nmse_fused).  Returns dY; the loss is ``self.loss``.
        ``bias_slabs`` (ops.slabsum.SlabBatch): queue the bias-gradient column reduction on it instead
        (the caller launches it in overwrite mode later in the step).  ``defer_loss`` (with
        ``bias_slabs``): no finish launch; ``self.pending_finish`` (a LossFinish) must be handed to a
        later launch of the step (ConvStackHIP.backward's ``loss_finish``), which forms loss and skip."""
        E, U, B = layout
        assert Y.is_cuda and self.rowoff is not None and Y.shape == (self.rows, self.cols) and self.rows == E * U * B
        self._check_labels(label)
        if perf is not None:
            self._check_labels(perf)
        m = rpc_mult or self.rpc_mult
        rpc = E * m if (B * E) % (E * m) == 0 else E
        chunks, gx = self.rows // rpc, self.cols // 1024
        dev = Y.device
        if getattr(self, "_fz", None) is None or self._fz[0] != (rpc, out_dtype):
            self._fz = ((rpc, out_dtype), torch.empty(chunks, self.cols, device=dev),
                        torch.empty(chunks * gx * E * 2, device=dev), torch.empty(self.S, 2, device=dev),
                        torch.empty(self.rows, self.cols, device=dev, dtype=out_dtype))
        _, colsum, part, dens, dY = self._fz
        rl = self._row_powers(label)
        rp = self._row_powers(perf) if perf is not None else None
        f = nat.fn(nat.hip_lib(), "qd_nmse_fused", [_p, _i, _p, _p, _p, _p, _p, _p, _i, _p, _p, _p, _p, _p, _p, _p,
                                                    _i, _i, _i, _i, _i, _f, _p, _i, _p])
        nat.check(f(nat.ptr(Y), int(Y.dtype == torch.bfloat16), nat.ptr(label),
                    nat.ptr(perf) if perf is not None else None, nat.ptr(self.rowoff), nat.ptr(rl),
                    nat.ptr(rp) if rp is not None else None, nat.ptr(dY), int(out_dtype == torch.bfloat16),
                    nat.ptr(colsum), nat.ptr(part), nat.ptr(dens), nat.ptr(bias_grad), nat.ptr(self.ss),
                    nat.ptr(self.loss), nat.ptr(self.skip), E, U, B, self.cols, rpc, loss_scale,
                    nat.ptr(rowden) if rowden is not None else None,
                    2 if defer_loss else int(bias_slabs is None), nat.stream_ptr(dev)),
                  "nmse_fused")
        self.pending_finish = None
        if defer_loss:
            assert bias_slabs is not None, "defer_loss needs the bias reduction queued elsewhere"
            self.pending_finish = LossFinish(nat.ptr(part), nat.ptr(dens), nat.ptr(self.ss), nat.ptr(self.loss),
                                             nat.ptr(self.skip) if self.skip is not None else None,
                                             gx, (B * E) // rpc, U, E)
        if bias_slabs is not None:
            bias_slabs.add(colsum, bias_grad, 1, chunks, self.cols)
        return dY

    def gemm_fused(self, A: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor], label: torch.Tensor,
                   perf: Optional[torch.Tensor], bias_grad: torch.Tensor, layout: Tuple[int, int, int],
                   rowden: torch.Tensor, loss_scale: float = 1.0, bias_slabs=None, defer_loss: bool = False,
                   cfg: int = 0, deq: Optional[torch.Tensor] = None, f8_out=None) -> torch.Tensor:
        """The FC forward GEMM with this loss as its epilogue (csrc/hip/gemm.hip qd_gemm_fwd_nmse): Y = A W^T
        + b is never written; dY (bf16), the error partials, the per-stream label powers and the bias
        gradient's per-tile column sums come out of the GEMM, then the same finish as ``fused`` (a launch,
        or ``pending_finish`` for a later launch of the step with ``defer_loss``; the bias column reduction
        queued on ``bias_slabs`` when given).  Returns dY; the loss is ``self.loss``.
        ``deq`` (2,) fp32: A and W are OCP e4m3 (torch.float8_e4m3fn) with these dequantisation scales
        (qd_gemm_fwd_nmse_f8, the fp8 estimator); the rest of the contract is unchanged.  ``f8_out`` (with
        ``deq``): (dY8 (M, N), dYt8 (N, M) or None, qs (1,), amax partials (4096,)) -- dY also written as e4m3,
        row-major (and transposed), for the fp8 backward GEMMs."""
        from .fc import gemm_tile_m
        E, U, B = layout
        M, K = A.shape
        N = W.shape[0]
        f8 = deq is not None
        assert A.is_cuda and self.rowoff is not None and M == self.rows == E * U * B and N == self.cols
        want = torch.float8_e4m3fn if f8 else torch.bfloat16
        assert A.dtype == W.dtype == want and A.is_contiguous() and W.is_contiguous()
        f8cfg = 0
        if f8:
            # (the e4m3 kernels have the cfg-0 tile; f8 cfg 1 = the MX-scaled MFMA when K allows)
            f8cfg = (2 if KNOBS.f8_producers else 1) if K % 256 == 0 else 0
            cfg = 0
        self._check_labels(label)
        if perf is not None:
            self._check_labels(perf)
        tm = gemm_tile_m(cfg)
        gx = N // 128
        dev = A.device
        if getattr(self, "_gz", None) is None or self._gz[0] != (tm, N):
            self._gz = ((tm, N), torch.empty(M, N, device=dev, dtype=torch.bfloat16),
                        torch.empty(M // 16 * gx * 2, device=dev), torch.empty(M // tm, N, device=dev),
                        torch.empty(self.S, 2, device=dev))
        _, dY, part, colsum, dens = self._gz
        if f8:
            f = nat.fn(nat.hip_lib(), "qd_gemm_fwd_nmse_f8", [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i,
                                                              _i, _i, _i, _i, _f, _i, _p, _p, _p, _p, _p])
            d8 = [None] * 4
            if f8_out is not None:
                dY8, dYt8, qs8, am8 = f8_out
                assert dY8.shape == (M, N) and dY8.element_size() == 1
                assert dYt8 is None or (dYt8.shape == (N, M) and dYt8.element_size() == 1)
                d8 = [nat.ptr(dY8), nat.ptr(dYt8) if dYt8 is not None else None, nat.ptr(qs8), nat.ptr(am8)]
            nat.check(f(nat.ptr(A), nat.ptr(W), nat.ptr(deq), nat.ptr(b) if b is not None else None, nat.ptr(label),
                        nat.ptr(perf) if perf is not None else None, nat.ptr(self.rowoff), nat.ptr(rowden),
                        nat.ptr(dY), nat.ptr(part), nat.ptr(colsum), nat.ptr(dens), M, N, K, E, U, B, loss_scale,
                        f8cfg, *d8, nat.stream_ptr(dev)), "gemm_fwd_nmse_f8")
        else:
            f = nat.fn(nat.hip_lib(), "qd_gemm_fwd_nmse", [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i,
                                                           _i, _i, _f, _i, _p])
            nat.check(f(nat.ptr(A), nat.ptr(W), nat.ptr(b) if b is not None else None, nat.ptr(label),
                        nat.ptr(perf) if perf is not None else None, nat.ptr(self.rowoff), nat.ptr(rowden),
                        nat.ptr(dY), nat.ptr(part), nat.ptr(colsum), nat.ptr(dens), M, N, K, E, U, B, loss_scale, cfg,
                        nat.stream_ptr(dev)), "gemm_fwd_nmse")
        self.pending_finish = None
        if defer_loss:
            assert bias_slabs is not None, "defer_loss needs the bias reduction queued elsewhere"
            self.pending_finish = LossFinish(nat.ptr(part), nat.ptr(dens), nat.ptr(self.ss), nat.ptr(self.loss),
                                             nat.ptr(self.skip) if self.skip is not None else None, gx, B // 16, U, E)
        else:
            fin = nat.fn(nat.hip_lib(), "qd_nmse_finish", [_p, _i, _p, _i, _i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p])
            nat.check(fin(nat.ptr(colsum), M // tm, nat.ptr(part), gx, B // 16, nat.ptr(dens), nat.ptr(bias_grad),
                          nat.ptr(self.ss), nat.ptr(self.loss), nat.ptr(self.skip) if self.skip is not None else None,
                          N, U, E, int(bias_slabs is None), nat.stream_ptr(dev)), "nmse_finish")
        if bias_slabs is not None:
            bias_slabs.add(colsum, bias_grad, 1, M // tm, N)
        return dY

    def __call__(self, Y, label, perf=None, out_dtype=torch.float32) -> Tuple[torch.Tensor, torch.Tensor]:
        self.sums(Y, label, perf)
        self.finalize()
        return self.loss, self.grad(Y, label, out_dtype)
