"""Capture invariants of the DP step's collective plumbing (parallel/dp.py GradBuckets, train/flagship_dp.py
DPPlan._dp_run), on the CPU with stub streams and events.

Round 4 found that a HIP graph capture in which a stream takes the SAME event as a dependency twice crashes
``hipStreamEndCapture`` (a duplicate edge, gpurun_out/r4_12; docs/CONCURRENCY.md "duplicate dependency
edges"), and that a capturing stream must never wait on an event recorded before the capture began.  This test
drives the real ``_dp_run`` through the ZeRO-1 and all-reduce plans, one to three steps per capture (the
one-graph plan), at simulated world 2 / 4 / 8, and checks both invariants on every ``wait_event``.  It fails if
GradBuckets._wait_on's dedupe is removed or a capture begins with a collective pending
(test_dedupe_is_what_keeps_it_clean)."""
import contextlib
import itertools
from types import SimpleNamespace

import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel import dp as dpmod
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext, GradBuckets
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship_dp import DPPlan


class Sim:
    """Stub HIP runtime: streams, events, a current-stream stack and a capture epoch."""

    def __init__(self):
        self.ids = itertools.count(1)
        self.epoch = 0            # capture number (0: not capturing)
        self.waits = []           # (stream id, event id, event epoch, epoch of the wait)
        self.main = self.Stream("main")
        self.stack = [self.main]

    def Stream(self, name):
        sim = self

        class S:
            def __init__(self):
                self.name, self.cuda_stream = name, next(sim.ids)

            def wait_event(self, ev):
                assert ev.recorded, "wait on an event that was never recorded"
                sim.waits.append((self.cuda_stream, ev.id, ev.epoch, sim.epoch))

            def wait_stream(self, other):   # (torch: records a fresh event on `other`, waits on it)
                e = sim.Event()
                e.record(other)
                self.wait_event(e)
        return S()

    def Event(self, **kw):
        sim = self

        class E:
            def __init__(self):
                self.id, self.recorded, self.epoch = next(sim.ids), False, None

            def record(self, stream=None):
                self.recorded, self.epoch = True, sim.epoch
                self.stream = stream if stream is not None else sim.stack[-1]
        return E()

    def current_stream(self, device=None):
        return self.stack[-1]

    @contextlib.contextmanager
    def stream(self, s):
        self.stack.append(s)
        try:
            yield
        finally:
            self.stack.pop()


class FakeComm:
    def __init__(self, log):
        self.log = log

    def all_reduce_(self, t, op="sum", stream=None):
        self.log.append(("all_reduce", stream.name))
        return t

    def reduce_scatter(self, out, inp, stream=None):
        self.log.append(("reduce_scatter", stream.name))
        return out

    def all_gather(self, out, inp, stream=None):
        self.log.append(("all_gather", stream.name))
        return out


def make_plan(sim, world, zero, one_graph=True):
    ctx = DistContext(rank=world - 1, world=world, backend="rccl", comm=FakeComm([]))
    ctx._comm_stream = sim.Stream("comm")
    n_conv, fc = 64, 64 * world
    grad = torch.zeros(n_conv + fc + 32)
    flat = torch.zeros_like(grad)
    bk = {"small": [grad[:n_conv]]}
    if not zero:
        bk["fc"] = [grad[n_conv:n_conv + fc]]
        bk["skip"] = [grad[-1:]]
    p = DPPlan()
    p.ctx, p.zero, p.buckets = ctx, zero, GradBuckets(ctx, bk)
    p._phases = p._stamps = None
    p.streams = {"fc": sim.Stream("fc"), "qsc": sim.Stream("qsc")}
    p.cfg = SimpleNamespace(dp_one_graph=one_graph, dp_qsc="g2")
    p.fc_region = (n_conv, n_conv + fc)
    p.hdce = SimpleNamespace(space=SimpleNamespace(grad=grad, flat=flat), fc_shadow=None)
    noop = lambda: None   # noqa: E731
    # (g2: the QSC branch forked onto its stream and joined back, as the real _dp_g2 does)

    def g2():
        qs = p.streams["qsc"]
        qs.wait_stream(sim.current_stream())
        sim.current_stream().wait_stream(qs)
    return p, (noop, noop, g2, noop, noop)


def capture(sim, plan, gs, k):
    """One graph capture of k DP steps (GraphedStep: guards first, then the body)."""
    plan.buckets.assert_quiescent()
    sim.epoch += 1
    first = len(sim.waits)
    for i in range(k):
        plan._dp_run(*gs, fence=i == k - 1, first=i == 0)
    assert not plan.buckets.pending
    return sim.waits[first:]


def check(waits):
    seen = set()
    for s, e, e_epoch, epoch in waits:
        assert (s, e) not in seen, "a stream waited twice on the same event inside one capture (duplicate edge)"
        seen.add((s, e))
        assert e_epoch == epoch, "a captured wait on an event recorded before the capture began"


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("zero", [True, False])
@pytest.mark.parametrize("k", [1, 2, 3])
def test_no_duplicate_or_stale_waits(world, zero, k, monkeypatch):
    sim = Sim()
    monkeypatch.setattr(torch.cuda, "current_stream", sim.current_stream)
    monkeypatch.setattr(torch.cuda, "stream", sim.stream)
    monkeypatch.setattr(torch.cuda, "Event", sim.Event)
    plan, gs = make_plan(sim, world, zero)
    for _ in range(3):   # consecutive captures (k-step sets of the same trainer)
        check(capture(sim, plan, gs, k))
    ops = [o for o, _ in plan.ctx.comm.log]
    per_step = ["reduce_scatter", "all_reduce", "all_gather"] if zero else ["all_reduce"] * 3
    assert ops == per_step * (3 * k)   # (one issue order per step on every rank)


def test_dedupe_is_what_keeps_it_clean(monkeypatch):
    """Without the dedupe the all-reduce plan waits twice on the FC collective's event from main (once as the
    ordering edge of the inline small-bucket all-reduce, once in wait()); a capture must not begin with a
    collective pending (assert_quiescent), whose wait would be on an event recorded before the capture."""
    sim = Sim()
    monkeypatch.setattr(torch.cuda, "current_stream", sim.current_stream)
    monkeypatch.setattr(torch.cuda, "stream", sim.stream)
    monkeypatch.setattr(torch.cuda, "Event", sim.Event)
    plan, gs = make_plan(sim, 4, zero=False)

    def no_dedupe(self, s, rec):
        if rec.stream.cuda_stream != s.cuda_stream:
            s.wait_event(rec.event)
    monkeypatch.setattr(GradBuckets, "_wait_on", no_dedupe)
    with pytest.raises(AssertionError, match="duplicate edge"):
        check(capture(sim, plan, gs, 1))
    monkeypatch.undo()

    sim = Sim()
    monkeypatch.setattr(torch.cuda, "current_stream", sim.current_stream)
    monkeypatch.setattr(torch.cuda, "stream", sim.stream)
    monkeypatch.setattr(torch.cuda, "Event", sim.Event)
    plan, gs = make_plan(sim, 4, zero=True)
    check(capture(sim, plan, gs, 1))
    plan.buckets.launch("small")   # (eager, outside any capture, and never waited for)
    with pytest.raises(RuntimeError, match="still pending"):
        capture(sim, plan, gs, 1)
    sim.epoch += 1                 # (had the guard let the capture begin, its wait would be on a stale event)
    n = len(sim.waits)
    plan.buckets.wait()
    with pytest.raises(AssertionError, match="before the capture began"):
        check(sim.waits[n:])


@pytest.mark.parametrize("n,k,lead,ramp,want", [
    (20, 10, 1, 4, [1, 4, 15]),          # the driver's window: the remainder rides in the last replay (3 boundaries)
    (300, 10, 1, 4, [1, 4] + [10] * 28 + [15]),
    (30, 10, 1, 4, [1, 4, 10, 15]),      # bench.py's settle run: warms every graph set the 20-step window uses
    (20, 10, 1, 0, [1, 10, 9]),          # ramp off: a merged 19-step graph exceeds one capture's data (fit 17)
    (3, 10, 1, 4, [1, 2]),
    (20, 1, 1, 4, [1] * 20),
    (25, 10, 0, 4, [10, 15]),
    (39, 10, 1, 4, [1, 4, 10, 10, 14]),
])
def test_replay_plan(n, k, lead, ramp, want):
    """FlagshipTrainer._reps: lead-in single step, one ramp replay, k-step replays, the remainder merged into the
    last one while the dataset holds that capture (else one remainder replay)."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import FlagshipTrainer
    fake = SimpleNamespace(cfg=SimpleNamespace(lead_in=lead, ramp=ramp), _k=lambda: k, store=SimpleNamespace(n=18000),
                           Bg=256)   # (fit = 18000 // (4 * 256) = 17 steps per capture)
    got = FlagshipTrainer._reps(fake, n)
    assert got == want and sum(got) == n
    # every graph set of the 20-step window is replayed by the 30-step settle run before it
    if n == 20 and k == 10:
        assert set(got) <= set(FlagshipTrainer._reps(fake, 30))


@pytest.mark.parametrize("a,c,g,n,want", [
    (0.03e-3, 0.06e-3, 0.39e-3, 20, None),     # a fast host: few replays
    (0.05e-3, 0.11e-3, 0.39e-3, 20, None),     # a slow one: no replay waits for its own submission
    (0.03e-3, 0.06e-3, 0.39e-3, 300, None),
    (0.0, 0.0, 0.39e-3, 20, [1, 17, 2]),        # free submission: the largest graphs (a tail of 2 is allowed)
])
def test_calibrated_replay_plan_never_waits_for_submission(a, c, g, n, want):
    """FlagshipTrainer._reps_calibrated: every replay's submission (a + c r, with the plan's margin) ends before the
    GPU runs out of the work queued ahead of it, sizes capped at what one capture holds."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import FlagshipTrainer as F
    fake = SimpleNamespace(cfg=SimpleNamespace(lead_in=1, ramp=4), _k=lambda: 10, store=SimpleNamespace(n=18000),
                           Bg=256, _sub_est=(a, c), _g_est=g, BOUNDARY_S=F.BOUNDARY_S, SUBMIT_MARGIN=F.SUBMIT_MARGIN)
    fake._reps_calibrated = lambda *args: F._reps_calibrated(fake, *args)
    got = F._reps(fake, n) if c > 0 else F._reps_calibrated(fake, n, 10, 17, (a, c), g)
    assert sum(got) == n and max(got) <= 17 and got[0] == 1
    A, C = F.SUBMIT_MARGIN * a, F.SUBMIT_MARGIN * c
    host = A + C
    gpu = host + g + F.BOUNDARY_S
    for r in got[1:]:
        host += A + C * r
        assert host <= gpu + 1e-12, got   # submitted before the GPU drained the replays queued ahead of it
        gpu += g * r + F.BOUNDARY_S
    if want is not None:
        assert got == want
    if n == 20 and c > 0:
        assert len(got) <= 4


def test_submission_fit():
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import FlagshipTrainer as F
    a, c = F._fit_submission([(1, 0.11e-3), (4, 0.29e-3), (10, 0.65e-3), (15, 0.95e-3), (1, 0.12e-3)])
    assert abs(c - 0.06e-3) < 0.005e-3 and 0.03e-3 < a < 0.07e-3
    assert F._fit_submission([(1, 2e-4), (1, 1e-4), (1, 3e-4)]) == (0.0, 2e-4)



def make_indep_plan(sim, world):
    """The DP plan with dp_qsc "indep" (DPPlan._dp_run_indep): stub kernels; the real stream / event / collective
    plumbing."""
    p, _ = make_plan(sim, world, zero=False)
    grad = p.hdce.space.grad
    p.buckets = GradBuckets(p.ctx, {"small": [grad[:48]], "q": [grad[48:64]], "fc": [grad[64:64 + 64 * world]],
                                    "skip": [grad[-1:]]})
    p.cfg = SimpleNamespace(dp_one_graph=True, dp_qsc="indep")
    noop = lambda *a, **k: None   # noqa: E731
    p._gather = noop
    p._qsc_branch = noop
    p._dp_g1b = noop
    p._dp_gf = noop
    p._adam_pack = lambda: None
    p._tail_pack_launch = noop
    p.tail_pack = False
    p._hgs = 1.0 / world
    p.qskip = p.hskip = None
    p.gat = None
    p.hstep = SimpleNamespace(hip=True, defer_dgrad=False, forward_conv_gathered=noop, dgrad=noop, backward_conv=noop)
    opt = SimpleNamespace(step=noop, bounds=[0, 1])
    p.hopt = p.qopt = opt
    return p


@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("k", [1, 2, 3])
def test_indep_dp_plan_capture_invariants(world, k, monkeypatch):
    """dp_qsc "indep" (round 6): the QSC chain's own bucket all-reduced from main at the next step's start (and at
    the replay's last step), waited for on the QSC stream -- no duplicate or stale waits over consecutive captures,
    and one collective order on every rank: [q of the previous step] skip, fc, small per step, q at the end."""
    sim = Sim()
    monkeypatch.setattr(torch.cuda, "current_stream", sim.current_stream)
    monkeypatch.setattr(torch.cuda, "stream", sim.stream)
    monkeypatch.setattr(torch.cuda, "Event", sim.Event)
    plan = make_indep_plan(sim, world)
    for _ in range(3):
        plan.buckets.assert_quiescent()
        sim.epoch += 1
        first = len(sim.waits)
        for i in range(k):
            plan._dp_run_indep(fence=i == k - 1, first=i == 0)
        assert not plan.buckets.pending
        check(sim.waits[first:])
    ops = [o for o, _ in plan.ctx.comm.log]
    assert ops == ["all_reduce"] * (3 * (4 * k))   # skip, fc, small per step + q once per step
    # the QSC bucket's collective is issued on the comm stream (forked from main), never from the qsc stream
    assert all(s != "qsc" for _, s in plan.ctx.comm.log)
