"""DP plan captured as ONE graph (RCCL collectives inside it) == the 5-graph DP plan, bit for bit.

    dp_one_graph.py OUT [zero|allreduce] [steps per one-graph replay] [g2|fwd|indep: the one-graph plan's QSC placement]

Run with QDML_FORCE_DIST=1 at world 1 on one GPU (a real RCCL process group of one rank: the
collectives are launched and captured exactly as at world N) or with N ranks.  Both plans train the
same model on the same batches for 6 steps; weights, moments and the bf16 FC shadow must agree
exactly (the graphs hold the same kernels in the same dependency order).  Then the one-graph trainer's
phase_times (clock stamps captured in a second copy of its graph) must give finite phases that fit in
the step."""
import faulthandler
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import (  # noqa: E402
    init_distributed, shutdown)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


def run(ctx, plan, one, k=1, steps=6, qsc="g2"):
    cfg = FlagshipConfig(n_qubits=8, batch=32, data_len=800, hip_graphs=True, dp_plan=plan,
                         split_graphs=True, dp_one_graph=one, steps_per_graph=k, dp_qsc=qsc)
    tr = FlagshipTrainer(cfg, ctx)
    tr.run(steps)
    tr.sync_master()
    torch.cuda.synchronize()
    return tr, len(tr.graphs), [t.cpu().clone() for t in tr.mutable_state()], tr.hloss.cpu().clone()


def main(out, plan="zero", k=1, qsc="g2"):
    faulthandler.enable()
    ctx = init_distributed("cuda")
    _, n5, s5, l5 = run(ctx, plan, False)
    print("five-graph plan done", flush=True)
    t1, n1, s1, l1 = run(ctx, plan, True, k, qsc=qsc)
    print("one-graph plan done", flush=True)
    same = [torch.equal(a, b) for a, b in zip(s5, s1)]
    ok = ctx.distributed and n5 == 5 and n1 == 1 and all(same) and torch.equal(l5, l1) and bool(torch.isfinite(l1).all())
    ph = t1.phase_times(3) if k == 1 else None
    ph_ok = ph is None or (all(v == v and 0.0 <= v < 1e3 for v in ph.values()) and ph["step"] > 0
                           and ph["g1"] <= ph["step"] and ph["g1"] + ph["g2"] <= ph["step"] + 1e-3)
    print("phases", ph, flush=True)
    with open(f"{out}.{ctx.rank}", "w") as f:
        f.write(f"{int(ok and ph_ok)} {n5} {n1} {''.join(str(int(x)) for x in same)} {l5.tolist()} {l1.tolist()}\n")
    shutdown()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "zero", int(sys.argv[3]) if len(sys.argv) > 3 else 1,
         sys.argv[4] if len(sys.argv) > 4 else "g2")
