"""The flagship trainer's data-parallel plan (world > 1; also world 1 with ``split_graphs``), as a mixin of
``train.flagship.FlagshipTrainer``: the step cut around its gradient collectives, the ZeRO-1 / all-reduce FC
update on its own stream, and per-phase timing (HIP events between the
5-graph plan's replays; device clock stamps captured inside the one-graph plan's graph).

Reference: torch.nn.DataParallel over 4 GPUs in the HDCE trainer (Runner_P128_QuantumNAT_onchipQNN.py:135-153,
SURVEY §2.4 C1-C7), re-designed as SPMD over RCCL: one process per GPU, bucketed collectives launched as soon
as their gradients are final and hidden behind the rest of the backward (see ``DPPlan._dp_run``).
"""
from __future__ import annotations

import ctypes

import torch

from .. import _native as nat
from ..utils.profiling import GraphedStep


class DPPlan:
    """Mixin: expects the FlagshipTrainer attributes (hstep, cstep, hopt, qopt, buckets, streams, ...)."""

    # -- the data-parallel plan (world > 1; also world 1 'serial' / split_graphs) ---------------
    #   g1 : gather, HDCE forward, NMSE, FC weight-gradient GEMM
    #        -> all-reduce 'skip' (HDCE NaN flag) and 'fc' (33.6 MB) start on RCCL's stream
    #   g2 : FC data-gradient GEMM, conv backward (+ wgrad side stream) and, on the qsc stream, the
    #        whole QSC forward/backward -- all of it hides the FC all-reduce
    #        -> all-reduce 'small' (conv/BN + QSC grads + the QSC NaN flag)
    #   gf : (fc stream) FC Adam once 'skip' + 'fc' arrived and g2's dgrad read the weight shadow,
    #        beside the 'small' all-reduce;   gr : (main) conv/BN Adam + QSC AdamW after 'small'
    def _qsc_fwd(self) -> bool:
        """(cfg.dp_qsc "fwd", one-graph plan) the QSC branch forks after the gather and joins in g2."""
        return self.cfg.dp_qsc == "fwd" and self.streams is not None and self._use_graphs

    def _dp_g1a(self) -> None:
        """gather + conv forward (reads no FC weight: overlaps the previous step's FC update)."""
        self._gather()
        if self._qsc_fwd():
            with self._fork(self.streams["qsc"]):
                self._qsc_branch(with_opt=False)
        self.hstep.defer_dgrad = self.hstep.hip
        if self.hstep.hip:
            self.hstep.forward_conv_gathered(self.gat)
        else:
            self._hdce_forward()

    def _dp_g1b(self) -> None:
        """FC forward, loss, FC weight gradient (on main: the FC collective waits for it first)."""
        if self.hstep.hip:
            loss = self.hstep.forward_fc_after_conv(self.store)
            if loss is not self.hloss:
                self.hloss.copy_(loss)

    def _dp_g1(self) -> None:
        self._dp_g1a()
        self._dp_g1b()

    def _dp_g2(self) -> None:
        """FC data gradient, conv backward and, on the qsc stream, the whole QSC forward/backward: the work
        that hides the FC gradient collective.  (World-1 rehearsal of the QSC placement: beside the conv
        backward 0.517 ms, beside the HDCE forward 0.492, split 0.557 -- this one leaves the most work behind
        the 33.6 MB FC collective, expected at 0.2-0.4 ms over xGMI at 2-8 ranks.)"""
        # NOTE the first node of a graph must sit on the capturing stream: a branch forked before any
        # node is a ROOT of the graph, and the HIP graph executor starts root nodes that it places on
        # its other queues without waiting for the work queued ahead of the graph launch (measured:
        # the QSC branch then read the previous step's gather output)
        if self.hstep.defer_dgrad:
            self.hstep.dgrad()
        if self._qsc_fwd():   # (forked in g1a: joined before the small bucket, which carries its gradients)
            self.hstep.backward_conv()
            self._join(("qsc",))
            return
        if self.streams is None:
            self.hstep.backward_conv()
            self._qsc_branch(with_opt=False)
            return
        with self._fork(self.streams["qsc"]):
            self._qsc_branch(with_opt=False)
        self.hstep.backward_conv()
        self._join(("qsc",))

    def _dp_gf(self) -> None:
        # (HDCE gradient scale _hgs: 1 / world for weak scaling, 1 for strong -- the ranks' losses are shares of one)
        if self.zero:   # this rank's shard of the FC region only
            self.hopt.step(grad_scale=self._hgs, skip=self.hskip, part=1 + self.ctx.rank)
        elif len(self.hopt.bounds) > 1:   # (unpartitioned -- serial world 1 -- gr steps everything)
            self.hopt.step(grad_scale=self._hgs, skip=self.hskip, part=1)

    def _dp_gr(self) -> None:
        pk = self._adam_pack()
        # (world-1 serial plan with adam_slabs: the update sums the step's gradient slabs itself)
        sl = self.hstep.take_slabs() if getattr(self, "adam_slabs", False) else None
        self.hopt.step(grad_scale=self._hgs, skip=self.hskip, part=0 if len(self.hopt.bounds) > 1 else None, pack=pk,
                       slabs=sl)
        if self.tail_pack and pk is None:
            self._tail_pack_launch()
        self.qopt.step(grad_scale=1.0 / self.ctx.world, skip=self.qskip)   # (QSC: the mean of equal-size parts)

    def _dp_run_indep(self, fence: bool = True, first: bool = True) -> None:
        """(cfg.dp_qsc "indep": the one-graph all-reduce plan) the world-1 step's independent chains inside the DP
        step.  The QSC chain gathers its own copy of the batch (device cursor cur[1]) and runs forward + backward
        on its stream without joining the HDCE chain; its gradients (bucket "q": QSC gradients + its NaN flag) are
        all-reduced at the START of the next step -- launched from main, as every captured collective must be
        (one launched from a forked stream crashed hipStreamEndCapture, scripts/probes/probe_rccl_capture.py) -- after
        main waits for the QSC chain of the previous step (long finished: ~150 us of QSC work against ~330 of HDCE
        work per step), and the QSC stream runs AdamW once it has landed, then the next QSC step.  The last step of
        a replay all-reduces and updates its own QSC gradients before the replay's join.  The HDCE chain has no QSC
        kernel and one cross-stream edge per step; every value is the serial step's (AdamW(i - 1) still runs before
        the QSC forward of step i).  ``fence``/``first`` as _dp_run.  (Reference DP site:
        Runner_P128_QuantumNAT_onchipQNN.py:135-153.)"""
        b = self.buckets
        main = torch.cuda.current_stream(self.ctx.device)
        q, fc = self.streams["qsc"], self.streams["fc"]

        def q_update():   # the QSC gradients of the step the qsc stream last ran: all-reduce, then AdamW
            main.wait_stream(q)
            b.launch("q")
            with torch.cuda.stream(q):
                b.wait(("q",))
                self.qopt.step(grad_scale=1.0 / self.ctx.world, skip=self.qskip)

        self._mark("start")
        if first:
            q.wait_stream(main)   # (a branch forked before any node would be a root of the graph)
        else:
            q_update()
        self._gather(classifier=False)
        with torch.cuda.stream(q):
            self._gather(hdce=False, classifier=True)
            self._qsc_branch(with_opt=False)
        self.hstep.defer_dgrad = self.hstep.hip
        if self.hstep.hip:
            self.hstep.forward_conv_gathered(self.gat)
        else:
            self._hdce_forward()
        if not first:   # (the previous step's FC update on the fc stream)
            main.wait_stream(fc)
        self._dp_g1b()
        b.launch("skip")
        b.launch("fc")
        if self.hstep.defer_dgrad:
            self.hstep.dgrad()
        self.hstep.backward_conv()
        b.launch("small", inline=True)
        fc.wait_stream(main)
        with torch.cuda.stream(fc):
            b.wait(("skip", "fc"))
            self._dp_gf()
        b.wait(("skip", "fc", "small"))
        pk = self._adam_pack()
        self.hopt.step(grad_scale=self._hgs, skip=self.hskip, part=0 if len(self.hopt.bounds) > 1 else None, pack=pk)
        if self.tail_pack and pk is None:
            self._tail_pack_launch()
        if fence:
            q_update()
            main.wait_stream(q)
            main.wait_stream(fc)
        b.clear()   # (every collective has been waited for by the stream that consumes it)
        self._mark("end")

    def _fc_weights_lp(self) -> torch.Tensor:
        """(ZeRO) the FC region's copy the forward / data gradient read: the bf16 shadow (GPU bf16),
        else the fp32 master weights themselves."""
        lo, hi = self.fc_region
        return self.hdce.fc_shadow if self.hdce.fc_shadow is not None else self.hdce.space.flat[lo:hi]

    def sync_master(self) -> None:
        """(ZeRO, bf16 shadow) each rank's fp32 FC master weights are current on its own shard only;
        all-gather them (checkpointing, cross-rank comparisons).  No-op otherwise."""
        if self.zero and self.ctx.distributed and self.hdce.fc_shadow is not None:
            lo, hi = self.fc_region
            self.buckets.launch_all_gather("master", self.hdce.space.flat[lo:hi])
            self.buckets.wait(("master",))
            self.buckets.pending.pop("master")   # (waited for by its only consumer: nothing stays in flight)
            if not self.buckets.pending:
                self.buckets.clear()

    def _mark(self, name: str, stream=None) -> None:
        """(phase timing) a HIP event on ``stream`` (default: current) under ``name``; while the stamped
        one-graph step is being captured, a clock-stamp node instead (csrc/hip/runtime.hip qd_stamp)."""
        if self._phases is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            self._phases[-1][name] = e
        elif self._stamps is not None:
            buf, slots = self._stamps
            i = slots.setdefault(name, len(slots))
            if i >= buf.numel():
                raise RuntimeError(f"phase stamp buffer full at {name!r}")
            s = stream if stream is not None else torch.cuda.current_stream(self.ctx.device)
            f = nat.fn(nat.hip_lib(), "qd_stamp", [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p])
            nat.check(f(nat.ptr(buf), i, ctypes.c_void_p(s.cuda_stream)), "qd_stamp")

    def _dp_run(self, g1a, g1b, g2, gf, gr, fence: bool = True, first: bool = True) -> None:
        """The DP step around the collectives.  RCCL runs every collective of the process group on one
        stream, in launch order: fc gradient (all-reduce, or reduce-scatter in the ZeRO plan), small
        bucket, (ZeRO) the shadow all-gather.
          allreduce : g1a g1b | AR fc | g2 | AR small | fc stream: FC Adam (whole FC) | main: conv/QSC Adam
          zero      : g1a g1b | RS fc | g2 | AR small | fc stream: FC Adam on 1/world, AG shadow | main: ...
        The FC update (fc stream) of step i overlaps step i+1's gather + conv forward (g1a): main waits
        for the fc stream only before g1b reads the FC weights.  ``fence``: main also waits for it at the
        end of the step (the last step of a run(), every step()): afterwards the state is complete."""
        b, zero = self.buckets, self.zero
        if self._phases is not None:
            self._phases.append({})
        self._mark("start")
        g1a()
        self._mark("g1a")
        main = torch.cuda.current_stream(self.ctx.device) if self.streams is not None else None
        if main is not None and not (self.cfg.dp_one_graph and first):
            # (the previous step's FC update, when not fenced; the one-graph plan always fences, and a
            # capturing stream must not wait on an event recorded outside the capture)
            main.wait_stream(self.streams["fc"])
        self._mark("fc_prev")
        g1b()
        self._mark("g1")
        lo, hi = self.fc_region
        if zero:
            b.launch_reduce_scatter("fc", self.hdce.space.grad[lo:hi])
        else:
            b.launch("skip")
            b.launch("fc")
        g2()
        self._mark("g2")
        # (main waits for the small bucket right away: its all-reduce runs inline on main -- ordered after the
        # FC collective -- instead of a fork / join through the comm stream, two cross-queue hops on the
        # step's critical path)
        b.launch("small", inline=True)
        b.launch("q", inline=True)   # (dp_qsc "indep" off the GPU streams: the QSC bucket beside the small one)
        fc_wait = ("fc", "small") if zero else ("skip", "fc")
        if self.streams is None:
            b.wait(fc_wait)
            gf()
            if zero:
                b.launch_all_gather("ag", self._fc_weights_lp())
            b.wait()
            gr()
            return
        fc = self.streams["fc"]
        if zero:
            # ZeRO: main takes the small bucket (collective + scatter-back) BEFORE forking the fc stream,
            # which needs its HDCE NaN flag: one stream owns each scatter-back, and the fc stream inherits
            # it through the fork (no second-waiter path across streams)
            b.wait(("small", "q"))
            fc_wait = ("fc",)
        fc.wait_stream(main)
        with torch.cuda.stream(fc):
            b.wait(fc_wait)
            self._mark("fc_ready", fc)
            gf()
            self._mark("gf", fc)
            if zero and self.cfg.dp_one_graph:
                # (captured: a collective launched from a forked stream crashes hipStreamEndCapture --
                # scripts/probes/probe_rccl_capture.py -- so main launches the all-gather; see below)
                pass
            elif zero:
                b.launch_all_gather("ag", self._fc_weights_lp())
                b.wait(("ag",))
                self._mark("ag", fc)
        # (allreduce plan: the HDCE NaN flag rides in the fc bucket -- wait for it before the conv Adam
        # reads it; free under RCCL, whose in-order stream finished fc before small)
        b.wait(("small", "q") if zero else ("skip", "fc", "small", "q"))
        self._mark("small_ready")
        og_ag = zero and self.cfg.dp_one_graph
        # the shadow all-gather from main once the shard is updated: before gr (it overlaps gr; the shard
        # Adam is 1/world of the FC) or after it (world 1: the whole-FC Adam on fc overlaps gr instead)
        ag_first = og_ag and self.ctx.world > 1
        if ag_first:
            main.wait_stream(fc)
            b.launch_all_gather("ag", self._fc_weights_lp())
        gr()
        self._mark("gr")
        if og_ag:
            if not ag_first:
                main.wait_stream(fc)
                b.launch_all_gather("ag", self._fc_weights_lp())
            b.wait(("ag",))
            self._mark("ag")
        b.clear()   # (every collective has been waited for by the stream that consumes it)
        if fence:
            main.wait_stream(fc)
        self._mark("end")

    def phase_times(self, steps: int):
        """Run ``steps`` DP steps with timers around the phases and return the mean milliseconds of each
        (diagnostic): g1a (gather + conv forward), fc_prev_wait, g1 (forward + FC wgrad), g2 (FC dgrad + conv
        backward + QSC, hiding the FC collective), fc_exposed (FC collective time left after g2),
        small_exposed, fc_adam, all_gather (ZeRO; the one-graph plan: its part left after gr),
        conv_qsc_adam, step.
          5-graph plan : HIP events between the graph replays (``run``: consecutive steps overlap, step =
                         start to the next step's start).
          one-graph    : a second capture of the one-step graph with a clock-stamp node at each phase
                         boundary on the phase's own stream, replayed ``steps`` times with a host sync after
                         each (step = its start to its fenced end).  The stamp nodes are extra graph nodes
                         (a few us each): the phases are the plan's shape, bench.py's timed run its speed.
        None for the world-1 single-chain plan and off the GPU."""
        if self.ctx.device.type != "cuda" or self.streams is None or self.cfg.dp_qsc == "indep":
            return None
        if len(self.graphs) == 5:
            rows, chained = self._event_rows(steps), True
        elif self.cfg.dp_one_graph and self._use_graphs and len(self.graphs) == 1 and \
                (self.ctx.world > 1 or self.cfg.split_graphs):
            rows, chained = self._stamped_rows(steps), False
        else:
            return None
        el = lambda r, a, b_: r[b_] - r[a]
        out = {"g1a": [], "fc_prev_wait": [], "g1": [], "g2": [], "fc_exposed": [], "small_exposed": [],
               "fc_adam": [], "all_gather": [], "conv_qsc_adam": [], "step": []}
        for i, r in enumerate(rows):
            out["g1a"].append(el(r, "start", "g1a"))
            out["fc_prev_wait"].append(el(r, "g1a", "fc_prev"))
            out["g1"].append(el(r, "start", "g1"))
            out["g2"].append(el(r, "g1", "g2"))
            out["fc_exposed"].append(max(0.0, el(r, "g2", "fc_ready")))
            out["small_exposed"].append(max(0.0, el(r, "g2", "small_ready")))
            out["fc_adam"].append(el(r, "fc_ready", "gf"))
            # (5-graph: the all-gather follows the shard Adam on the fc stream; one-graph: main launches it
            # beside gr, and only what is left of it after gr is on the critical path)
            ag_from = "gf" if chained else "gr"
            out["all_gather"].append(max(0.0, el(r, ag_from, "ag")) if "ag" in r else 0.0)
            out["conv_qsc_adam"].append(el(r, "small_ready", "gr"))
            nxt = rows[i + 1]["start"] if chained and i + 1 < len(rows) else r["end"]
            out["step"].append(nxt - r["start"])
        return {k: sum(v) / len(v) for k, v in out.items()}

    def _event_rows(self, steps: int):
        """(5-graph plan) ``run(steps)`` with HIP events at the phase boundaries -> per-step {phase: ms}
        relative to the first step's start."""
        self._phases = []
        try:
            self.run(steps)
            torch.cuda.synchronize(self.ctx.device)
            rows = self._phases
        finally:
            self._phases = None
        t0 = rows[0]["start"]
        return [{k: t0.elapsed_time(e) for k, e in r.items()} for r in rows]

    def _stamped_rows(self, steps: int):
        """(one-graph plan) the one-step graph captured again with clock stamps (see ``_mark``), replayed
        ``steps`` times -> per-step {phase: ms} on the device clock."""
        dev = self.ctx.device
        buf = torch.zeros(32, dtype=torch.int64, device=dev)
        self._stamps = (buf, {})
        gs = [GraphedStep(lambda: self._dp_run(self._dp_g1a, self._dp_g1b, self._dp_g2, self._dp_gf, self._dp_gr),
                          enabled=True, guards=(self.buckets.assert_quiescent,))]
        try:
            self._capture_set(gs, 1, preserve=True)
            slots = dict(self._stamps[1])
        finally:
            self._stamps = None
        khz = ctypes.c_int(0)
        f = nat.fn(nat.hip_lib(), "qd_wallclock_khz", [ctypes.c_int, ctypes.POINTER(ctypes.c_int)])
        nat.check(f(dev.index if dev.index is not None else torch.cuda.current_device(), ctypes.byref(khz)),
                  "qd_wallclock_khz")
        if khz.value <= 0:
            raise RuntimeError(f"device wall clock rate {khz.value} kHz")
        rows = []
        try:
            for _ in range(steps):
                self.next_batch(1)
                gs[0]()
                torch.cuda.synchronize(dev)
                t = buf.tolist()
                rows.append({n: (t[i] - t[slots["start"]]) / khz.value for n, i in slots.items()})
        finally:
            del gs   # (the stamped graph and its pool)
        return rows
