"""The capture-safe RCCL failure detector (parallel/watchdog.py).  CPU: a fake communicator
stands in for RcclComm (async_error / close(abort)), so stalls and asynchronous errors can be injected."""
import os
import subprocess
import sys
import textwrap
import threading
import time

import pytest

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel import watchdog as wdm
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeComm:
    def __init__(self):
        self.err = 0
        self.aborted = threading.Event()
        self.closed_with = None

    def async_error(self):
        return self.err

    def close(self, abort=False):
        self.closed_with = abort
        if abort:
            self.aborted.set()


class Clock:
    def __init__(self):
        self.t = 100.0

    def __call__(self):
        return self.t


def test_check_once_stall_error_and_disarm():
    c, clk = FakeComm(), Clock()
    w = wdm.CommWatchdog(c, rank=3, timeout_s=10, clock=clk)
    assert w.check_once() is None
    clk.t += 9
    assert w.check_once() is None
    w.heartbeat("epoch 2")
    clk.t += 9.5
    assert w.check_once() is None            # (the heartbeat reset the age)
    clk.t += 1.0
    msg = w.check_once()
    assert msg is not None and "epoch 2" in msg and "10" in msg
    w.arm(False)                             # disarmed: quiet is not a stall ...
    clk.t += 1000
    assert w.check_once() is None
    c.err = 5                                # ... but an asynchronous error still is
    assert "asynchronous error 5" in w.check_once()


def test_thread_fires_on_stall_and_aborts():
    c = FakeComm()
    got = []
    w = wdm.CommWatchdog(c, rank=1, timeout_s=0.3, poll_s=0.05, on_fail=lambda code, msg: got.append((code, msg)))
    w.heartbeat("train step")
    t0 = time.monotonic()
    w.start()
    assert c.aborted.wait(5.0), "the watchdog did not abort a stalled communicator"
    w._thread.join(5.0)
    assert time.monotonic() - t0 < 3.0
    assert c.closed_with is True
    assert got and got[0][0] == wdm.EXIT_STALL and "rank 1" in got[0][1] and "train step" in got[0][1]


def test_thread_fires_on_async_error():
    c = FakeComm()
    got = []
    w = wdm.CommWatchdog(c, rank=0, timeout_s=1e6, poll_s=0.05, on_fail=lambda code, msg: got.append(code)).start()
    time.sleep(0.2)
    assert not got
    c.err = 2
    assert c.aborted.wait(5.0)
    w._thread.join(5.0)
    assert got == [wdm.EXIT_COMM_ERROR]


def test_heartbeats_keep_it_quiet_and_stop_joins():
    c = FakeComm()
    got = []
    w = wdm.CommWatchdog(c, rank=0, timeout_s=0.25, poll_s=0.02, on_fail=lambda code, msg: got.append(code)).start()
    ctx = DistContext(watchdog=w)
    for i in range(40):   # 0.8 s of work with a completed sync point every 20 ms
        time.sleep(0.02)
        ctx.heartbeat(f"step {i}")
    w.stop()
    assert not w._thread.is_alive()
    assert not got and not c.aborted.is_set()


def test_capture_pauses_async_error_polling():
    """While a HIP graph is being captured nothing but the heartbeat age is checked (no RCCL call at all)."""
    c = FakeComm()
    c.err = 7
    w = wdm.CommWatchdog(c, rank=0, timeout_s=1e6)
    with wdm.capturing():
        assert w.check_once() is None
    assert "asynchronous error 7" in w.check_once()


def test_stall_inside_a_capture_window_still_fires():
    """the capture window pauses only the RCCL call -- a stall (a peer dead during the warm-up
    collectives or the pre-capture sync) is still detected."""
    c, clk = FakeComm(), Clock()
    w = wdm.CommWatchdog(c, rank=2, timeout_s=5, clock=clk)
    w.heartbeat("graph capture")
    with wdm.capturing():
        clk.t += 6
        msg = w.check_once()
    assert msg is not None and "graph capture" in msg


def test_graphed_step_capture_window_is_the_graph_block_only(monkeypatch):
    """GraphedStep.capture: the eager warm-ups run OUTSIDE capturing() (a stall there is visible), and the
    heartbeat is bumped right before and after the graph block."""
    import torch
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.utils import profiling
    seen = []

    class G:
        def reset(self):
            pass

    @__import__("contextlib").contextmanager
    def fake_graph(g, **kw):
        seen.append(("graph", wdm._capture_depth))
        yield

    class S:
        def wait_stream(self, other):
            pass

    monkeypatch.setattr(torch.cuda, "Stream", lambda *a, **k: S())
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: S())
    monkeypatch.setattr(torch.cuda, "stream", lambda s: __import__("contextlib").nullcontext())
    monkeypatch.setattr(torch.cuda, "CUDAGraph", G)
    monkeypatch.setattr(torch.cuda, "graph", fake_graph)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    beats = []
    monkeypatch.setattr(wdm, "heartbeat", lambda phase=None: beats.append(phase))
    gs = profiling.GraphedStep(lambda: seen.append(("fn", wdm._capture_depth)), warmup=2)
    gs.capture()
    assert seen == [("fn", 0), ("fn", 0), ("graph", 1), ("fn", 1)]
    assert beats == ["graph capture", "graph replay"] and wdm._capture_depth == 0
    gs.close()
    with pytest.raises(RuntimeError, match="after close"):
        gs()


def test_module_heartbeat_and_disarmed_reach_the_running_watchdog():
    c, clk = FakeComm(), Clock()
    w = wdm.CommWatchdog(c, rank=0, timeout_s=5, poll_s=3600, clock=clk).start()
    try:
        assert wdm._active is w
        clk.t += 4
        wdm.heartbeat("epoch 3")
        clk.t += 4
        assert w.check_once() is None                # (the module-level heartbeat reached it)
        with wdm.disarmed("data generation"):
            clk.t += 1000
            assert w.check_once() is None            # host-only phase: no stall
        assert w._armed and w.check_once() is None   # re-armed with a fresh heartbeat
        clk.t += 6
        assert "data generation" in w.check_once()
    finally:
        w.stop()
    assert wdm._active is None


def test_pg_timeout_env_reaches_the_watchdog_timeout(monkeypatch):
    """QDML_PG_TIMEOUT is the default of init_distributed's timeout (rendezvous AND the watchdog), not
    only bench.py's."""
    import inspect
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel import dp
    monkeypatch.setenv("QDML_PG_TIMEOUT", "1234")
    assert dp.resolve_timeout() == 1234.0 and dp.resolve_timeout(7) == 7.0
    assert inspect.signature(dp.init_distributed).parameters["timeout_s"].default is None


def test_hung_abort_is_not_waited_for():
    class Stuck(FakeComm):
        def close(self, abort=False):
            time.sleep(30)
    got = []
    w = wdm.CommWatchdog(Stuck(), rank=0, timeout_s=0.1, poll_s=0.05, abort_grace_s=0.3,
                         on_fail=lambda code, msg: got.append(code)).start()
    t0 = time.monotonic()
    while not got and time.monotonic() - t0 < 5:
        time.sleep(0.05)
    assert got == [wdm.EXIT_STALL] and time.monotonic() - t0 < 3


def test_stalled_process_exits_nonzero():
    """The real failure path: a process whose sync point never completes ends itself with EXIT_STALL within the
    timeout (os._exit from the watchdog thread while the main thread is blocked), after aborting the
    communicator."""
    script = textwrap.dedent("""
        import sys, time
        sys.path.insert(0, %r)
        from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.watchdog import CommWatchdog
        class C:
            def async_error(self): return 0
            def close(self, abort=False): print("abort=%%s" %% abort, file=sys.stderr, flush=True)
        w = CommWatchdog(C(), rank=4, timeout_s=0.5, poll_s=0.1).start()
        w.heartbeat("all_reduce of the epoch loss")
        time.sleep(60)   # a peer died: this host sync never returns
        print("unreachable", flush=True)
    """) % REPO
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=30)
    assert p.returncode == wdm.EXIT_STALL, (p.returncode, p.stderr)
    assert time.monotonic() - t0 < 20
    assert "rank 4" in p.stderr and "all_reduce of the epoch loss" in p.stderr and "abort=True" in p.stderr
    assert "unreachable" not in p.stdout


def test_normal_process_unaffected():
    script = textwrap.dedent("""
        import sys, time
        sys.path.insert(0, %r)
        from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.watchdog import CommWatchdog
        class C:
            def async_error(self): return 0
            def close(self, abort=False): print("closed abort=%%s" %% abort, flush=True)
        c = C()
        w = CommWatchdog(c, rank=0, timeout_s=0.5, poll_s=0.05).start()
        for i in range(20):
            time.sleep(0.05)
            w.heartbeat("epoch %%d" %% i)
        w.stop()
        c.close()
    """) % REPO
    p = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=30)
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip() == "closed abort=False"


def test_backend_selection(monkeypatch):
    """QDML_DIST_BACKEND: rccl (default on GPUs), gloo, or torch's own ProcessGroupNCCL kept as a fallback
    (torch_nccl); anything else is an error, and the GPU backends refuse to start without a GPU."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel import dp
    monkeypatch.setattr(dp, "_CTX", None)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("QDML_DIST_BACKEND", "bogus")
    with pytest.raises(ValueError, match="rccl, gloo or torch_nccl"):
        dp.init_distributed("cpu")
    for b in ("torch_nccl", "rccl", "nccl"):
        monkeypatch.setenv("QDML_DIST_BACKEND", b)
        with pytest.raises(RuntimeError, match="needs a GPU"):
            dp.init_distributed("cpu")
    assert dp._CTX is None
