"""Tracing / profiling helpers: roctx ranges, HIP-event timers, HIP-graph step capture.

Reference: wall-clock only -- ``time.time()`` around QSC training (R:437-440) and a
timestamp per HDCE epoch (R:173).  Here:
  * ``trace_range(name)`` -- roctx range (visible in ``rocprofv3 --marker-trace``) when
                         libroctx64 is loadable, otherwise a no-op;
  * ``EventTimer``    -- HIP-event phase timing without host syncs inside the step;
  * ``GraphedStep``   -- captures a whole training step (gather, forward, backward,
                         optimizer) into one HIP graph after a warm-up on a side
                         stream and replays it; removes per-kernel launch overhead,
                         which dominates this small-model workload.
"""
from __future__ import annotations

import atexit
import contextlib
import ctypes
import os
from typing import Callable, Dict, List, Optional, Sequence

import torch

_roctx = None


def _load_roctx():
    global _roctx
    if _roctx is None:
        _roctx = False
        for p in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(p)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx


@contextlib.contextmanager
def trace_range(name: str):
    lib = _load_roctx() if os.environ.get("QDML_ROCTX", "1") == "1" else False
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


class EventTimer:
    """Accumulates per-phase GPU time with HIP events; ``summary()`` syncs once."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self.events: Dict[str, List] = {}

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        yield
        e.record()
        self.events.setdefault(name, []).append((s, e))

    def summary(self) -> Dict[str, float]:
        if not self.enabled:
            return {}
        torch.cuda.synchronize()
        return {k: sum(s.elapsed_time(e) for s, e in v) / len(v) for k, v in self.events.items()}


_GRAVEYARD: list = []   # graph executables of closed / dropped GraphedSteps, destroyed at exit (or a safe point)
# When a parked executable is destroyed.  "exit" (default): at interpreter exit only.  Round 6's native crash
# report (profiles/r6_11b_bench_forced_segfault.txt) put the recurring host segfault of hipGraphLaunch (rounds 5
# and 6, multi-stream graphs) inside the HIP runtime's graph scheduling (hip_graph_internal.cpp: a node pointer
# read as 0x21, then +0x1a8 dereferenced), and every occurrence followed the destruction of OTHER graph executables
# in the same process (earlier tests' trainers, bench.py's losing plan candidates).  Their device memory stays
# reserved until exit (a few GB per flagship trainer: HBM has room).  "sync": destroy at the next safe point.
GRAPH_RELEASE = os.environ.get("QDML_GRAPH_RELEASE", "exit")


def release_dropped_graphs(final: bool = False) -> None:
    """Destroy the parked graph executables (GraphedStep.close / __del__) after a device sync -- at exit
    (``final``), or at a safe point when QDML_GRAPH_RELEASE=sync: never while a capture is running (a sync there
    invalidates it), never from a finaliser."""
    if not _GRAVEYARD or (GRAPH_RELEASE != "sync" and not final):
        return
    if torch.cuda.is_available():
        if torch.cuda.is_current_stream_capturing():
            return
        torch.cuda.synchronize()
    while _GRAVEYARD:
        _GRAVEYARD.pop().reset()


atexit.register(release_dropped_graphs, True)


class GraphedStep:
    """Capture ``fn`` (which reads/writes only static tensors) into a HIP graph.

    ``fn`` is run ``warmup`` times on a side stream first (allocator + library
    handle warm-up, as graph capture requires), then captured once; ``__call__``
    replays.  With ``enabled=False`` it simply calls ``fn`` (eager).
    """

    WARMUP = 3

    def __init__(self, fn: Callable[[], None], enabled: bool = True, warmup: Optional[int] = None, pool=None,
                 capture_stream: Optional["torch.cuda.Stream"] = None, capture_error_mode: str = "global",
                 guards: Sequence[Callable[[], None]] = ()):
        """``capture_stream``: the stream the graph is captured on (e.g. a high-priority one, so the
        nodes of its chain keep that priority over side branches forked from lower-priority streams).
        ``guards``: checks run right before the capture begins (each raises if the process is not
        quiescent, e.g. a gradient collective still pending)."""
        self.capture_stream = capture_stream
        self.capture_error_mode = capture_error_mode
        self.guards = list(guards)
        self.fn = fn
        self.enabled = enabled and torch.cuda.is_available()
        self.warmup = self.WARMUP if warmup is None else warmup
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.pool = pool

    def capture(self) -> None:
        from ..parallel.watchdog import capturing, heartbeat
        release_dropped_graphs()   # (a safe point: no capture or replay of ours is running)
        # eager warm-ups (real collectives under the DP plans) stay visible to the failure detector: only the
        # capture itself pauses it (a peer that dies during a warm-up or the pre-capture sync is a stall)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                self.fn()
        torch.cuda.current_stream().wait_stream(s)
        self.pre_capture()
        heartbeat("graph capture")
        g = torch.cuda.CUDAGraph()
        if self.capture_stream is not None:
            self.capture_stream.wait_stream(torch.cuda.current_stream())
        with capturing():
            with torch.cuda.graph(g, pool=self.pool, stream=self.capture_stream,
                                  capture_error_mode=self.capture_error_mode):
                self.fn()
        heartbeat("graph replay")
        self.graph = g

    def close(self) -> None:
        """Retire the step: the graph executable is parked (destroyed at exit, or -- QDML_GRAPH_RELEASE=sync -- right
        here after a device sync, so no replay of it can still be running when HIP destroys it).  (Rounds 5 and 6: a
        host segfault in a later hipGraphLaunch of another graph after executables were destroyed, see
        GRAPH_RELEASE.)  Idempotent; calling the step afterwards raises."""
        g, self.graph = self.graph, None
        self.enabled = False
        self.fn = None   # (breaks the trainer -> graph set -> step -> bound method cycle)
        if g is not None:
            _GRAVEYARD.append(g)
        release_dropped_graphs()

    def __del__(self) -> None:
        # no HIP call here: the garbage collector can run this in the middle of another graph's capture or replay
        # (round 6: the round-5 hipGraphLaunch segfault recurred in a replay after earlier tests' graphs were
        # dropped by collection, profiles/r6_11a_pytest_segfault.log).  The executable is parked and destroyed at exit
        # (release_dropped_graphs; QDML_GRAPH_RELEASE).
        try:
            if self.graph is not None:
                _GRAVEYARD.append(self.graph)
                self.graph = None
        except Exception:   # (interpreter shutdown)
            pass

    def pre_capture(self) -> None:
        """The capture starts from a quiescent process: every warm-up kernel and collective has finished
        on the device (host sync), and every guard passes.  (Round 3's captured-collective abort: a thread
        other than the capturing one touched an event of a warm-up collective while the capture ran --
        docs/CONCURRENCY.md "captured collectives".)"""
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        for g in self.guards:
            g()

    def __call__(self) -> None:
        if not self.enabled:
            if self.fn is None:
                raise RuntimeError("GraphedStep used after close()")
            self.fn()
            return
        if self.graph is None:
            self.capture()
        self.graph.replay()
