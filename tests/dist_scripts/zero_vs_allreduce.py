"""ZeRO-1 FC optimizer plan == all-reduce plan, bit for bit (gloo, CPU or one shared GPU).

    zero_vs_allreduce.py OUT [cpu|cuda]

Both plans train the same model on the same rank-local batches for a few steps; the ZeRO plan's
master weights are all-gathered (sync_master) and compared with the all-reduce plan's.  With two
ranks a sum of two floats is order-free, so the reduce-scatter and the all-reduce agree exactly."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import (  # noqa: E402
    init_distributed, shutdown)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


def run(ctx, plan, device, steps=3):
    if device == "cuda":
        # (QDML_STREAM_MODE: diagnosis of the GPU rehearsal -- serial takes the QSC branch off its stream)
        cfg = FlagshipConfig(n_qubits=8, batch=32, data_len=800, hip_graphs=True, dp_plan=plan,
                             use_quantumnat=False, stream_mode=os.environ.get("QDML_STREAM_MODE", "dagq"))
    else:
        cfg = FlagshipConfig(n_qubits=4, batch=4, data_len=40, hip_graphs=False, dtype="fp32", dp_plan=plan,
                             use_quantumnat=False)
    tr = FlagshipTrainer(cfg, ctx)
    for _ in range(steps):
        tr.step()
    tr.sync_master()
    if device == "cuda":
        torch.cuda.synchronize()
    n = tr.hdce.space.n_real
    lo, hi = tr.fc_region
    return (tr.zero, tr.hdce.space.flat[:n].cpu().clone(), tr.qspace.flat.cpu().clone(),
            tr.hdce.fc_shadow.cpu().clone() if tr.hdce.fc_shadow is not None else None, tr.hloss.cpu().clone())


def main(out, device="cpu"):
    ctx = init_distributed(device)
    # (QDML_ZV_PLANS="allreduce,allreduce" etc.: the same plan twice -- run-to-run determinism)
    pa, pz = os.environ.get("QDML_ZV_PLANS", "allreduce,zero").split(",")
    za, fa, qa, sa, la = run(ctx, pa, device)
    zz, fz, qz, sz, lz = run(ctx, pz, device)
    checks = {"plans": za == (pa == "zero") and zz == (pz == "zero"), "hdce": torch.equal(fa, fz), "qsc": torch.equal(qa, qz),
              "loss": torch.equal(la, lz)}
    if sa is not None:
        checks["shadow"] = torch.equal(sa[:fa.numel() - (fa.numel() - sa.numel())], sz[:sa.numel()])
    g = [torch.empty_like(fz) for _ in range(ctx.world)]
    dist.all_gather(g, fz)
    checks["ranks"] = all(torch.equal(g[0], x) for x in g[1:])   # every rank holds the same weights
    ok = all(checks.values())
    diff = float((fa - fz).abs().max())
    failed = ",".join(k for k, v in checks.items() if not v) or "-"
    with open(f"{out}.{ctx.rank}", "w") as f:
        f.write(f"{int(ok)} {diff} {failed} qdiff={float((qa - qz).abs().max())} loss={la.tolist()}/{lz.tolist()}\n")
    shutdown()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "cpu")
