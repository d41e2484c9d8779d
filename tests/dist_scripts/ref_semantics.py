"""DataParallel semantics (dp_semantics="reference"): N ranks each take their part of ONE global batch per
stream; the result must equal a single process training on the whole global batch.

    ref_semantics.py OUT [world_1_reference]

Classical SC (BN-free): every parameter after one epoch equals the 1-rank run within fp32 tolerance.
HDCE: the run completes in lockstep (per-replica BatchNorm, as DataParallel, makes its parameters differ
from a full-batch BN run by design), with rank-identical parameters and BN buffers.  At world 3 the global
batch of 8 splits 3/3/2 and at world 8 the partial last batch (6 rows) leaves two ranks with no rows: both
must still run every collective in lockstep."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train import runner as rmod  # noqa: E402


def main(out):
    ws = os.path.join(os.path.dirname(out), f"ws_{os.environ.get('WORLD_SIZE', '1')}")
    kw = dict(device="cpu", data_len=60, batch_size_DML=8, n_epochs=1, dtype="fp32", hip_graphs=False, workspace=ws,
              log_jsonl="", dp_semantics="reference", optimizer="adam")
    r = rmod.Y2HRunner(**kw)
    sc = r.train_SC_P128()
    flat = torch.cat([p.detach().reshape(-1) for p in sc.parameters()])
    m = r.train_Conv_Linear_of_HDCE()
    h = m.space.flat.clone()
    ctx = r._context()
    same = True
    if ctx.world > 1:
        # weights AND the BN running buffers (rank 0's, broadcast before evaluation / checkpointing) agree
        for t in (h, torch.cat(m.run_mean + m.run_var), m._nbt.double()):
            g = [torch.empty_like(t) for _ in range(ctx.world)]
            dist.all_gather(g, t)
            same = same and all(torch.equal(g[0], x) for x in g[1:])
    torch.save({"sc": flat, "hdce_loss": torch.tensor(r.train_HDCE_losses), "sc_loss": torch.tensor(r.train_SC_losses)},
               f"{out}.{ctx.rank}.pt")
    with open(f"{out}.{ctx.rank}", "w") as f:
        f.write(f"{int(same)} {r.train_HDCE_losses[-1]} {r.train_SC_losses[-1]}\n")


if __name__ == "__main__":
    main(sys.argv[1])
