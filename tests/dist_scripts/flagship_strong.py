"""Strong scaling of the flagship trainer (FlagshipConfig.scaling="strong": the reference's DataParallel split of
ONE global batch per stream, R:144-148), against a 1-process trainer on the whole global batch built in the same
process.

    flagship_strong.py OUT

Checked per rank, over 3 steps: (1) this rank's conv input is exactly rows [rank * b, (rank + 1) * b) of every
stream's global batch (the DataParallel scatter); (2) the NMSE denominators are the global batch's; (3) the QSC
(no BatchNorm) weights equal the 1-process run's within fp32 tolerance -- the ranks' mean of per-part mean
losses is the global mean; (4) every parameter is bit-identical across ranks.  (The HDCE normalises with per-rank
BatchNorm statistics, as DataParallel's replicas do, so its weights differ from a full-batch BN run by design.)"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import (  # noqa: E402
    DistContext, init_distributed, shutdown)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


def same_on_all_ranks(t):
    g = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(g, t)
    return all(torch.equal(g[0], x) for x in g[1:])


def main(out):
    ctx = init_distributed("cpu")
    bg = 8
    kw = dict(n_qubits=4, batch=bg, data_len=60, hip_graphs=False, dtype="fp32", use_quantumnat=False,
              dp_plan="allreduce")
    ref = FlagshipTrainer(FlagshipConfig(**kw), DistContext(device=torch.device("cpu")))   # 1 process, whole batch
    tr = FlagshipTrainer(FlagshipConfig(scaling="strong", **kw), ctx)
    b, off, U = tr.B, ctx.rank * tr.B, tr.U
    ok = [b * ctx.world == bg, torch.equal(tr.perm, ref.perm), same_on_all_ranks(tr.perm.float())]
    for _ in range(3):
        c = tr.cursor
        tr.step()
        ref.step()
        gl = tr.perm[c:c + bg]
        den = torch.stack([tr.store.Hlabel.index_select(1, gl).pow(2).sum((1, 2)),
                           tr.store.Hperf.index_select(1, gl).pow(2).sum((1, 2))], 1)
        ok.append(torch.allclose(tr.gat.den_global, den, rtol=1e-6))
        part = ref.gat.x1.view(U, bg, *ref.gat.x1.shape[1:])[:, off:off + b]
        ok.append(torch.equal(tr.gat.x1.view(U, b, *tr.gat.x1.shape[1:]), part))
        ok.append(same_on_all_ranks(torch.cat([tr.hdce.space.flat, tr.qspace.flat])))
    qa, qb = (torch.cat([sp.flat[sp.slice_of(p)] for p in sp.params]) for sp in (tr.qspace, ref.qspace))
    dq = float((qa - qb).abs().max())
    ok.append(torch.allclose(qa, qb, rtol=1e-4, atol=1e-6))
    with open(f"{out}.{ctx.rank}", "w") as f:
        f.write(f"{int(all(ok))} {dq} {[int(x) for x in ok]}\n")
    shutdown()


if __name__ == "__main__":
    main(sys.argv[1])
