"""Step-plan experiments without touching the product code: alternative capture structures of the world-1
dagq step, as subclasses of FlagshipTrainer; prints ms/step for each (same timing contract as bench.py:
warm-up, capture, settle, then a timed window).  Run under rocprofv3 --kernel-trace with PLAN=<name> to get
the timeline of one plan.

    python scripts/probes/r4_plan_probe.py [steps]          # PLAN=all (default) or one plan name
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


class HdceFirst(FlagshipTrainer):
    """HDCE chain captured before the QSC branch (the QSC forks from an event after the gather)."""

    def _step_body(self):
        self._gather()
        ev = torch.cuda.Event()
        ev.record()
        self._hdce_graph()
        qs = self.streams["qsc"]
        qs.wait_event(ev)
        with torch.cuda.stream(qs):
            self._qsc_branch(with_opt=True)
        self._join(("qsc",))


class JoinLast(FlagshipTrainer):
    """The round-3 plan: the QSC branch joins AFTER the HDCE chain's last node (the Adam), so the next step's
    gather has two parents on two queues.  (Round 4 ships the join before the Adam, measured here as
    'join_first' before it became the default: profiles/r4_08_plan_probe.txt.)"""

    def _step_body(self):
        self._gather()
        with self._fork(self.streams["qsc"]):
            self._qsc_branch(with_opt=True)
        self._hdce_graph()
        self._join(("qsc",))


class ForkAfter(FlagshipTrainer):
    """As shipped, but the QSC branch's nodes are created AFTER the HDCE chain's first conv launch(es) -- its only
    dependency is still the gather (an event recorded right after it).  The graph executor keeps a node's first
    created child on the parent's queue: shipped, that child is the QSC branch and the conv forward hops queues
    (~13 us after the gather, profiles/r4_14_step_timeline.md); here the conv forward is the first child."""
    FORK_AT = "conv1"

    def _step_body(self):
        self._gather()
        ev = torch.cuda.Event()
        ev.record()
        qs = self.streams["qsc"]

        def hook(stage):
            if stage == self.FORK_AT:
                qs.wait_event(ev)
                with torch.cuda.stream(qs):
                    self._qsc_branch(with_opt=True)

        self.hstep.stage_hook = hook
        try:
            self._hdce_forward()
        finally:
            self.hstep.stage_hook = None
        self.hstep.backward_conv()
        self._join(("qsc",))
        self._hdce_update()


class ForkAfterConv2(ForkAfter):
    FORK_AT = "conv2"


class ForkAfterConv3(ForkAfter):
    FORK_AT = "conv3"


def adam_grid(g):
    class AdamGrid(FlagshipTrainer):
        """As shipped, the HDCE update launched on at most ``g`` workgroups (default 2048)."""

        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.hopt.max_grid[0] = g
    return AdamGrid


def knobs(**kw):
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS

    class WithKnobs(FlagshipTrainer):
        """As shipped, built under other knobs.KNOBS values (restored after construction)."""

        def __init__(self, *a, **k):
            old = {n: getattr(KNOBS, n) for n in kw}
            for n, v in kw.items():
                setattr(KNOBS, n, v)
            try:
                super().__init__(*a, **k)
            finally:
                for n, v in old.items():
                    setattr(KNOBS, n, v)
    return WithKnobs


class HdceOnly(FlagshipTrainer):
    """(diagnostic, not a training step) the HDCE chain alone: what the concurrent QSC branch costs it."""

    def _step_body(self):
        self._gather()
        self._hdce_forward()
        self.hstep.backward_conv()
        self._hdce_update()


class QscOnly(FlagshipTrainer):
    """(diagnostic) the QSC branch alone, on the capturing stream."""

    def _step_body(self):
        self._gather()
        self._qsc_branch(with_opt=True)


PLANS = {"hdce_only": HdceOnly, "qsc_only": QscOnly,
         "fused_loss6": knobs(hand_gemm="fwd,wgrad,dgrad", gemm_cfg="6,1,2"),
         "fused_loss1": knobs(hand_gemm="fwd,wgrad,dgrad", gemm_cfg="1,1,2"),
         "adam1024": adam_grid(1024), "adam1536": adam_grid(1536), "shipped": FlagshipTrainer, "hdce_first": HdceFirst, "join_last": JoinLast, "fork_conv1": ForkAfter,
         "fork_conv2": ForkAfterConv2,
         "fork_conv3": ForkAfterConv3,
         # the FC weight's Adam in the weight-gradient GEMM's epilogue (round 3 measured it slower with the
         # round-3 plan; re-measured after the join move), on the shipped and the 8-wave K-split wgrad tile
         "fused_adam": (FlagshipTrainer, {"fused_fc_adam": True}),
         "fused_adam_w2": (knobs(gemm_cfg="6,2,2"), {"fused_fc_adam": True})}


def run(cls, steps):
    cls, cfgkw = cls if isinstance(cls, tuple) else (cls, {})
    ctx = DistContext(device=torch.device("cuda", 0))
    tr = cls(FlagshipConfig(steps_per_graph=10, pilot_num=int(os.environ.get("PILOT", "128")),
                            n_qubits=int(os.environ.get("QUBITS", "8")), **cfgkw), ctx)
    tr.run(20)
    tr.prepare(steps)
    tr.run(30)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run(steps)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, tr


def main(steps):
    want = os.environ.get("PLAN", "all")
    names = list(PLANS) if want == "all" else want.split(",")
    for rnd in range(int(os.environ.get("ROUNDS", "2")) if len(names) > 1 else 1):
        for n in names:
            ms, tr = run(PLANS[n], steps)
            print(f"{n:12s} {ms:.4f} ms/step  loss {tr.hloss.tolist()[0]:.5f}", flush=True)
            del tr
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 300)
