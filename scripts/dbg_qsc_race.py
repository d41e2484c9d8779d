"""Debug: is the fused QSC step bit-reproducible when other kernels run concurrently?

Runs QSCStepHIP forward+backward on fixed inputs alone (reference), then repeatedly with a heavy
GEMM workload on a second stream, and reports which intermediate buffers differ bitwise.

    PYTHONPATH=. python scripts/dbg_qsc_race.py [trials]
"""
import sys

import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import FlagshipConfig, FlagshipTrainer


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    ctx = DistContext(device=torch.device("cuda", 0))
    tr = FlagshipTrainer(FlagshipConfig(hip_graphs=False, stream_mode="serial", batch=256), ctx)
    h = tr.cstep.hip
    tr.next_batch()
    tr._gather()
    torch.cuda.synchronize()
    names = ["angles", "E", "dE", "dang", "dpre", "p2", "p1s", "c1", "c2", "preslab", "qslab", "psave", "wnoisy"]

    def run_once():
        h.noise_ctr.zero_()
        tr._qsc_branch(with_opt=False)

    def snap():
        out = {n: getattr(h, n).clone() for n in names if getattr(h, n, None) is not None}
        out["grad"] = tr.qspace.grad.clone()
        out["loss"] = h.loss.clone()
        return out

    run_once()
    torch.cuda.synchronize()
    ref = snap()
    run_once()
    torch.cuda.synchronize()
    again = snap()
    print("alone, twice:", [n for n in ref if not torch.equal(ref[n], again[n])], flush=True)
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    side = torch.cuda.Stream()
    bad = {}
    for t in range(trials):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(6):
                a = (a @ a).clamp_(-1, 1)
        run_once()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        cur = snap()
        diff = [n for n in ref if not torch.equal(ref[n], cur[n])]
        for n in diff:
            bad[n] = bad.get(n, 0) + 1
        print("trial", t, "differ:", diff, {n: float((ref[n].float() - cur[n].float()).abs().max()) for n in diff}, flush=True)
    print("SUMMARY", bad)


if __name__ == "__main__":
    main()
