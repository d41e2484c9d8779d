"""Capture-safe failure detector for the RCCL communicator.

Reference: the reference has no failure handling at all -- ``nn.DataParallel`` in one process
(Runner_P128_QuantumNAT_onchipQNN.py:135-153) simply raises or hangs.  Torch's process group had a
watchdog thread, but it polls HIP events, and an event query from another thread while a HIP graph
is being captured aborts the capture (round 3, docs/CONCURRENCY.md "captured collectives") -- which
is why the framework runs its own communicator (parallel/comm.py) without one.

This watchdog makes NO HIP calls.  One daemon thread per rank:
  * watches a host-side heartbeat that the training loop bumps at every completed host sync point
    (DistContext.barrier / all_reduce_ / max_vector, the end of an epoch, an evaluation, a checkpoint);
  * polls ``ncclCommGetAsyncError`` every ``poll_s`` seconds (a host-side read of the communicator's
    error state, the call NCCL/RCCL documents for watchdogs);
  * on an asynchronous error, or a heartbeat older than ``timeout_s`` while armed, it logs the rank, the
    phase that stalled and for how long, calls ``ncclCommAbort`` (``RcclComm.close(abort=True)``: the
    stuck RCCL kernels return, so the blocked host sync can finish) and ends the process with a
    non-zero code (``os._exit``, never an exec).  An abort that itself hangs is not waited for beyond
    ``abort_grace_s``.

The default timeout is ``QDML_PG_TIMEOUT`` (600 s), the same knob that bounds the rendezvous.
"""
from __future__ import annotations

import contextlib
import os
import sys
import threading
import time
from typing import Callable, Optional

EXIT_STALL = 75       # (EX_TEMPFAIL) a peer stopped answering: the job can be restarted from its checkpoint
EXIT_COMM_ERROR = 76  # RCCL reported an asynchronous error

_capture_depth = 0   # HIP graph captures in progress in this process (utils.profiling.GraphedStep)
_active: Optional["CommWatchdog"] = None   # the running watchdog of this process (one communicator per rank)


@contextlib.contextmanager
def capturing():
    """Around a HIP graph capture -- the ``torch.cuda.graph`` block only, not its eager warm-ups: the watchdog makes
    no RCCL call meanwhile (belt and braces: the async-error read is host-only, but a capture is exactly where round
    3's process-group watchdog broke things).  The heartbeat-age check keeps running: it reads host memory only."""
    global _capture_depth
    _capture_depth += 1
    try:
        yield
    finally:
        _capture_depth -= 1


def heartbeat(phase: Optional[str] = None) -> None:
    """Bump the running watchdog's heartbeat, if there is one (a host sync point completed; ``phase``: what runs
    next).  Cheap and safe to call from any host code."""
    wd = _active
    if wd is not None:
        wd.heartbeat(phase)


@contextlib.contextmanager
def disarmed(phase: str):
    """Around host-only work that may legitimately outlast the timeout with no collective in flight (data
    generation, rank-0-only checkpointing / evaluation while the other ranks wait at the next barrier): the stall
    check is off meanwhile (async errors still fire), and re-armed with a fresh heartbeat afterwards."""
    wd = _active
    if wd is None:
        yield
        return
    wd.arm(False)
    wd.heartbeat(phase)
    try:
        yield
    finally:
        wd.arm(True)


class CommWatchdog:
    """``comm``: an object with ``async_error() -> int`` and ``close(abort: bool)`` (RcclComm, or a test
    double).  ``on_fail(code, message)``: what to do after the abort (default: print and ``os._exit``)."""

    def __init__(self, comm, rank: int, timeout_s: float, poll_s: float = 2.0, abort_grace_s: float = 10.0,
                 on_fail: Optional[Callable[[int, str], None]] = None, clock: Callable[[], float] = time.monotonic):
        self.comm, self.rank = comm, rank
        self.timeout_s, self.poll_s, self.abort_grace_s = float(timeout_s), float(poll_s), float(abort_grace_s)
        self.on_fail = on_fail or _exit_process
        self.clock = clock
        self._lock = threading.Lock()
        self._beat = clock()
        self._phase = "init"
        self._armed = True
        self._stop = threading.Event()
        self.fired: Optional[str] = None   # the failure message once the watchdog has fired
        self._thread = threading.Thread(target=self._run, name=f"qdml-comm-watchdog-{rank}", daemon=True)

    # -- training-loop side (cheap: a lock and two stores) -------------------------------------------
    def start(self) -> "CommWatchdog":
        global _active
        self._thread.start()
        _active = self
        return self

    def heartbeat(self, phase: Optional[str] = None) -> None:
        """A host sync point completed (``phase``: what runs next, for the stall report)."""
        with self._lock:
            self._beat = self.clock()
            if phase is not None:
                self._phase = phase

    def arm(self, armed: bool = True) -> None:
        """Disarmed, a long quiet period (host-only work between jobs) is not a stall; async errors still fire."""
        with self._lock:
            self._armed = armed
            self._beat = self.clock()

    def stop(self) -> None:
        global _active
        if _active is self:
            _active = None
        self._stop.set()
        if self._thread.is_alive() and threading.current_thread() is not self._thread:
            self._thread.join(timeout=self.poll_s + 1.0)

    # -- watchdog thread ------------------------------------------------------------------------------
    def check_once(self) -> Optional[str]:
        """One poll: the failure message, or None.  (Exposed for tests; the thread calls it every poll_s.)"""
        if _capture_depth == 0:   # (no RCCL call while a graph is being captured; the stall check below stays)
            try:
                err = int(self.comm.async_error())
            except Exception as e:   # (a destroyed communicator while shutting down is not a failure)
                if self._stop.is_set():
                    return None
                return f"ncclCommGetAsyncError raised {e!r}"
            if err != 0:
                return f"RCCL asynchronous error {err}"
        with self._lock:
            age, phase, armed = self.clock() - self._beat, self._phase, self._armed
        if armed and age > self.timeout_s:
            return f"no host sync point completed for {age:.1f} s (timeout {self.timeout_s:.0f} s) in phase '{phase}'"
        return None

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            msg = self.check_once()
            if msg is None:
                continue
            self._fire(msg)
            return

    def _fire(self, msg: str) -> None:
        code = EXIT_COMM_ERROR if msg.startswith(("RCCL", "nccl")) else EXIT_STALL
        self.fired = f"[qdml watchdog] rank {self.rank}: {msg}; aborting the communicator"
        print(self.fired, file=sys.stderr, flush=True)
        # ncclCommAbort unblocks the RCCL kernels a stuck stream waits on; it may itself block on a dead peer,
        # so it runs on a helper thread that is waited for at most abort_grace_s
        t = threading.Thread(target=self._abort, daemon=True)
        t.start()
        t.join(self.abort_grace_s)
        if t.is_alive():
            print(f"[qdml watchdog] rank {self.rank}: ncclCommAbort did not return in {self.abort_grace_s:.0f} s",
                  file=sys.stderr, flush=True)
        self.on_fail(code, self.fired)

    def _abort(self) -> None:
        try:
            self.comm.close(abort=True)
        except Exception as e:
            print(f"[qdml watchdog] rank {self.rank}: abort raised {e!r}", file=sys.stderr, flush=True)


def _exit_process(code: int, msg: str) -> None:
    sys.stderr.flush()
    sys.stdout.flush()
    os._exit(code)


def default_timeout_s() -> float:
    return float(os.environ.get("QDML_PG_TIMEOUT", "600"))
