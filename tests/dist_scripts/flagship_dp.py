"""World-N flagship trainer: ranks stay bit-identical; a NaN on ONE rank makes every rank skip the step
(the NaN-guard flags ride in the gradient buckets).

    flagship_dp.py OUT [cpu|cuda]

cpu: gloo, eager.  cuda: the real DP plan (4 HIP graphs, side streams, bucketed async all-reduces)
with QDML_DIST_BACKEND=gloo so several ranks can share one GPU (RCCL needs a GPU per rank)."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import (  # noqa: E402
    init_distributed, shutdown)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


def flat_all(tr):
    tr.sync_master()   # (ZeRO plan: each rank's fp32 FC master is current on its own shard only)
    tr.buckets.assert_quiescent()   # (nothing left in flight: a later graph capture would refuse to start)
    ts = [tr.hdce.space.flat, tr.qspace.flat]
    if tr.hdce.fc_shadow is not None:   # the bf16 weights the forward reads
        ts.append(tr.hdce.fc_shadow.float())
    return torch.cat(ts)


def same_on_all_ranks(t):
    t = t.cpu()   # (gloo gathers host tensors)
    g = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(g, t)
    return all(torch.equal(g[0], x) for x in g[1:])


def main(out, device="cpu"):
    ctx = init_distributed(device)
    plan = os.environ.get("QDML_DP_PLAN", "zero")
    if device == "cuda":
        cfg = FlagshipConfig(n_qubits=8, batch=32, data_len=800, hip_graphs=True, dp_plan=plan)
    else:
        cfg = FlagshipConfig(n_qubits=4, batch=4, data_len=40, hip_graphs=False, dtype="fp32", dp_plan=plan)
    tr = FlagshipTrainer(cfg, ctx)
    ok = [same_on_all_ranks(flat_all(tr))]
    dbg = os.environ.get("QDML_DBG") == "1"
    for i in range(2):
        tr.step()
        ok.append(same_on_all_ranks(flat_all(tr)))
        if dbg:
            print(ctx.rank, "step", i, "same", ok[-1], "skip", tr.skip_flags().tolist(), "h", float(tr.hdce.space.flat.double().sum()),
                  "q", float(tr.qspace.flat.double().sum()), "hg", float(tr.hdce.space.grad.double().sum()),
                  "steps", tr.hopt.step_t.tolist(), tr.qopt.step_t.tolist(), flush=True)
    before = flat_all(tr).clone()
    # NaN injected into rank 1's data only
    if ctx.rank == 1:
        tr.store.Yp.fill_(float("nan"))
    tr.step()
    after = flat_all(tr)
    skipped = torch.equal(before, after)
    ok.append(same_on_all_ranks(after))
    with open(f"{out}.{ctx.rank}", "w") as f:
        f.write(f"{int(all(ok))} {int(skipped)} {float(tr.skip_flags().sum().item())}\n")
    shutdown()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "cpu")
