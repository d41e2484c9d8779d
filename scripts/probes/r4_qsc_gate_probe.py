"""Step-plan probe for the large-circuit configurations: the QSC branch's backward half gated on the HDCE loss.

At P256 / 12 qubits the 253-VGPR simulator backward (qsim_big_bwd_kernel<12>, ~440 us) starts right after the
simulator forward and fills every SIMD's register file while the HDCE chain runs its memory-bound NMSE pass,
which then takes ~220 us instead of ~35 (profiles/r4_11_p256_timeline.md).  'gate_loss' forks the QSC forward
half after the gather as shipped, but the backward half waits (one cross-queue edge) for the HDCE loss: the
simulator backward then overlaps the FC gradient GEMMs and the conv backward instead.

    r4_qsc_gate_probe.py PILOT QUBITS [steps] [rounds]      (PLAN=<name> for one plan, e.g. under rocprofv3)
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


class GateLoss(FlagshipTrainer):
    def _step_body(self):
        self._gather()
        qs = self.streams["qsc"]
        with self._fork(qs):
            self.cstep.forward_part(self.gat.xq, self.labels)
        orig = self.hstep._fc_backward

        def fc_backward(dY, A, W):
            ev = torch.cuda.Event()
            ev.record()
            qs.wait_event(ev)
            with torch.cuda.stream(qs):
                q = self.cstep.backward_part(self.gat.xq, slabs=self.qslabs if self.cstep.writes_grads else None)
                if self.cstep.writes_grads:
                    self.qslabs.launch(accumulate=False, stream=nat.stream_ptr(self.ctx.device))
                if q is not self.qloss:
                    self.qloss.copy_(q)
                self.qopt.step(grad_scale=1.0, skip=self.qskip)
            orig(dY, A, W)

        self.hstep._fc_backward = fc_backward
        try:
            self._hdce_forward()
        finally:
            self.hstep._fc_backward = orig
        self.hstep.backward_conv()
        self._join(("qsc",))
        self._hdce_update()


PLANS = {"shipped": FlagshipTrainer, "gate_loss": GateLoss}


def main():
    pilot = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    qubits = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    only = os.environ.get("PLAN")
    names = [only] if only else list(PLANS)
    ctx = DistContext(device=torch.device("cuda", 0))
    store = None
    for r in range(rounds):
        for n in names:
            tr = PLANS[n](FlagshipConfig(pilot_num=pilot, n_qubits=qubits, steps_per_graph=10), ctx, store=store)
            store = tr.store
            tr.run(20)
            tr.prepare(steps)
            tr.run(30)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.run(steps)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            print(f"round {r} P{pilot} q{qubits} {n:10s} {ms:.4f} ms/step  loss {float(tr.hloss[0]):.5f} "
                  f"qloss {float(tr.qloss.reshape(-1)[0]):.5f}", flush=True)
            del tr
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
