"""RCCL communicator (GPU collective backend), over the native wrapper ``csrc/hip/comm.hip``.

Reference: DataParallel's implicit NCCL broadcast / reduce / peer copies from one process
(Runner_P128_QuantumNAT_onchipQNN.py:135-153).

MI355X design: one process per GPU, one RCCL communicator per process.  Every collective is
stream-ordered on the stream the caller names (default: the current stream) -- no process-group
progress thread, no per-collective events or work objects.  A collective issued while that stream
is being captured becomes a node of the HIP graph; its ordering against compute is the graph's
(or the streams') own edges.  The communicator id is exchanged through the job's c10d store
(torchrun's agent store or a TCPStore at MASTER_ADDR:MASTER_PORT).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from .. import _native as nat

# dtype / op codes of csrc/hip/comm.hip
_DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float64: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5}
_OPS = {"sum": 0, "max": 1, "min": 2}


class CommError(RuntimeError):
    pass


def rccl_path() -> str:
    """The librccl torch itself links (one RCCL per process); QDML_RCCL_LIB overrides."""
    p = os.environ.get("QDML_RCCL_LIB")
    if p:
        return p
    cand = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return cand if os.path.exists(cand) else "librccl.so.1"


def _lib():
    lib = nat.hip_lib()
    f = nat.fn(lib, "qd_comm_load", [ctypes.c_char_p])
    st = f(rccl_path().encode())
    if st != 0:
        raise CommError(f"cannot bind RCCL from {rccl_path()}")
    es = getattr(lib, "qd_comm_error_string")
    es.argtypes, es.restype = [ctypes.c_int], ctypes.c_char_p
    return lib


def _check(lib, st: int, what: str) -> None:
    if st != 0:
        raise CommError(f"{what}: RCCL status {st} ({lib.qd_comm_error_string(st).decode(errors='replace')})")


def rccl_version() -> int:
    lib = _lib()
    v = ctypes.c_int(0)
    _check(lib, nat.fn(lib, "qd_comm_version", [ctypes.POINTER(ctypes.c_int)])(ctypes.byref(v)), "ncclGetVersion")
    return v.value


def new_unique_id() -> bytes:
    lib = _lib()
    n = nat.fn(lib, "qd_comm_id_bytes", [])()
    buf = (ctypes.c_uint8 * n)()
    _check(lib, nat.fn(lib, "qd_comm_unique_id", [ctypes.c_void_p, ctypes.c_int])(buf, n), "ncclGetUniqueId")
    return bytes(buf)


class _StdoutToStderr:
    """fd-level redirect of stdout to stderr: RCCL prints its version banner on stdout at initialisation, and a
    benchmark's stdout carries exactly one JSON line (bench.py)."""

    def __enter__(self):
        import sys
        sys.stdout.flush()
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        import sys
        sys.stdout.flush()
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


class RcclComm:
    """One rank of an RCCL communicator on ``device``.  ``store``: a c10d Store shared by the ranks
    (the communicator id travels through it under ``key``)."""

    def __init__(self, rank: int, world: int, device: torch.device, store, key: str = "qdml_rccl_id"):
        self.rank, self.world, self.device = rank, world, device
        self.lib = _lib()
        L = self.lib
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        self._ar = nat.fn(L, "qd_comm_all_reduce", [vp, vp, vp, sz, i, i, vp])
        self._rs = nat.fn(L, "qd_comm_reduce_scatter", [vp, vp, vp, sz, i, i, vp])
        self._ag = nat.fn(L, "qd_comm_all_gather", [vp, vp, vp, sz, i, vp])
        self._bc = nat.fn(L, "qd_comm_broadcast", [vp, vp, vp, sz, i, i, vp])
        self._gs = nat.fn(L, "qd_comm_group_start", [])
        self._ge = nat.fn(L, "qd_comm_group_end", [])
        if rank == 0:
            with _StdoutToStderr():
                uid = new_unique_id()
            store.set(key, uid)
        else:
            uid = store.get(key)   # (blocks until rank 0 has published it)
        n = nat.fn(L, "qd_comm_id_bytes", [])()
        if len(uid) != n:
            raise CommError(f"communicator id of {len(uid)} bytes, expected {n}")
        self.comm = ctypes.c_void_p()
        with torch.cuda.device(device), _StdoutToStderr():
            st = nat.fn(L, "qd_comm_init", [ctypes.POINTER(ctypes.c_void_p), i, ctypes.c_char_p, i])(
                ctypes.byref(self.comm), world, uid, rank)
        _check(L, st, f"ncclCommInitRank(rank {rank} of {world})")
        cnt = ctypes.c_int(0)
        _check(L, nat.fn(L, "qd_comm_count", [vp, ctypes.POINTER(ctypes.c_int)])(self.comm, ctypes.byref(cnt)),
               "ncclCommCount")
        if cnt.value != world:
            raise CommError(f"communicator has {cnt.value} ranks, expected {world}")

    # -- helpers -------------------------------------------------------------------------------------
    def _stream(self, stream: Optional[torch.cuda.Stream]) -> ctypes.c_void_p:
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return ctypes.c_void_p(s.cuda_stream)

    def _dt(self, t: torch.Tensor) -> int:
        if not t.is_cuda or not t.is_contiguous():
            raise CommError("RCCL collectives take contiguous device tensors")
        try:
            return _DTYPES[t.dtype]
        except KeyError:
            raise CommError(f"unsupported dtype {t.dtype}") from None

    # -- collectives (stream-ordered; nothing waits on the host) --------------------------------------
    def all_reduce_(self, t: torch.Tensor, op: str = "sum", stream=None, out: Optional[torch.Tensor] = None):
        """In place (or into ``out``) sum / max / min over ranks."""
        dst = t if out is None else out
        if dst.numel() != t.numel() or dst.dtype != t.dtype:
            raise CommError("all_reduce: out must match the input")
        st = self._ar(self.comm, nat.ptr(t), nat.ptr(dst), t.numel(), self._dt(t), _OPS[op], self._stream(stream))
        _check(self.lib, st, "ncclAllReduce")
        return dst

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        """``out`` = this rank's block ``inp.view(world, -1)[rank]`` of the sum over ranks."""
        if inp.numel() != out.numel() * self.world or inp.dtype != out.dtype:
            raise CommError(f"reduce_scatter: {inp.numel()} elements in, {out.numel()} x {self.world} out")
        st = self._rs(self.comm, nat.ptr(inp), nat.ptr(out), out.numel(), self._dt(inp), _OPS[op], self._stream(stream))
        _check(self.lib, st, "ncclReduceScatter")
        return out

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, stream=None) -> torch.Tensor:
        """``out.view(world, -1)[r]`` = rank r's ``inp``."""
        if out.numel() != inp.numel() * self.world or inp.dtype != out.dtype:
            raise CommError(f"all_gather: {inp.numel()} elements in, {out.numel()} out at world {self.world}")
        st = self._ag(self.comm, nat.ptr(inp), nat.ptr(out), inp.numel(), self._dt(inp), self._stream(stream))
        _check(self.lib, st, "ncclAllGather")
        return out

    def broadcast_(self, t: torch.Tensor, src: int = 0, stream=None) -> torch.Tensor:
        st = self._bc(self.comm, nat.ptr(t), nat.ptr(t), t.numel(), self._dt(t), src, self._stream(stream))
        _check(self.lib, st, "ncclBroadcast")
        return t

    def group(self):
        """Context manager: the collectives issued inside launch as ONE fused RCCL operation."""
        comm = self

        class _G:
            def __enter__(self_):
                _check(comm.lib, comm._gs(), "ncclGroupStart")

            def __exit__(self_, *exc):
                _check(comm.lib, comm._ge(), "ncclGroupEnd")
                return False
        return _G()

    # -- health / teardown ----------------------------------------------------------------------------
    def async_error(self) -> int:
        e = ctypes.c_int(0)
        _check(self.lib, nat.fn(self.lib, "qd_comm_async_error", [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)])(
            self.comm, ctypes.byref(e)), "ncclCommGetAsyncError")
        return e.value

    def check(self) -> None:
        """Raise if RCCL recorded an asynchronous error (a peer died, a network failure)."""
        e = self.async_error()
        if e != 0:
            raise CommError(f"RCCL asynchronous error {e} ({self.lib.qd_comm_error_string(e).decode(errors='replace')})")

    def close(self, abort: bool = False) -> None:
        if self.comm:
            st = nat.fn(self.lib, "qd_comm_destroy", [ctypes.c_void_p, ctypes.c_int])(self.comm, 1 if abort else 0)
            self.comm = ctypes.c_void_p()
            _check(self.lib, st, "ncclCommDestroy")
