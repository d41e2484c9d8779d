"""The framework's RCCL communicator (parallel/comm.py) on one GPU, world 1 (QDML_FORCE_DIST=1): every
collective eager and captured in a HIP graph, then a runner HDCE run whose steps capture the bucketed
gradient all-reduces (hip_graphs on) against the same run eager.

    rccl_world1.py OUT WORKSPACE
writes "1" to OUT.0 when every check passes (else the failed checks)."""
import faulthandler
import os
import sys
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import (  # noqa: E402
    GradBuckets, init_distributed, shutdown)


def collectives(ctx):
    comm, dev, fails = ctx.comm, ctx.device, []
    x = torch.arange(1000, dtype=torch.float32, device=dev)
    y = torch.empty_like(x)
    comm.all_reduce_(x, out=y)
    comm.all_reduce_(x, "max")
    bf = torch.ones(64, dtype=torch.bfloat16, device=dev)
    comm.all_reduce_(bf)
    d = torch.full((3,), 2.5, dtype=torch.float64, device=dev)
    comm.all_reduce_(d, "min")
    rs = torch.empty(500, device=dev)
    comm.reduce_scatter(rs, torch.arange(500, dtype=torch.float32, device=dev))
    ag = torch.empty(500, device=dev)
    comm.all_gather(ag, torch.arange(500, dtype=torch.float32, device=dev))
    bc = torch.full((7,), 3.0, device=dev)
    comm.broadcast_(bc)
    a1, a2 = torch.ones(10, device=dev), torch.ones(20, device=dev)
    with comm.group():
        comm.all_reduce_(a1)
        comm.all_reduce_(a2)
    torch.cuda.synchronize()
    ref = torch.arange(1000, dtype=torch.float32, device=dev)
    checks = {"ar_out": torch.equal(y, ref), "ar_max": torch.equal(x, ref), "bf16": bool((bf == 1).all()),
              "f64_min": bool((d == 2.5).all()), "rs": torch.equal(rs, ref[:500]), "ag": torch.equal(ag, ref[:500]),
              "bcast": bool((bc == 3).all()), "group": bool((a1 == 1).all() and (a2 == 1).all())}
    fails += [k for k, v in checks.items() if not v]
    comm.check()
    # the bucket pattern captured in a graph (fork to the comm stream, join back), replayed twice
    g1 = torch.zeros(1 << 16, device=dev)
    g2, g3 = torch.zeros(100, device=dev), torch.zeros(3, device=dev)
    full = torch.zeros(4096, device=dev)
    bk = GradBuckets(ctx, {"big": [g1], "small": [g2, g3]})

    def body():
        g1.add_(1.0)
        g2.add_(2.0)
        g3.add_(3.0)
        full.add_(1.0)
        bk.launch("big")
        bk.launch("small", inline=True)   # (on the capturing stream, after "big": the DP step's small bucket)
        bk.launch_reduce_scatter("rs", full)
        bk.wait()
        bk.launch_all_gather("ag", full)
        bk.wait()

    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream(dev).wait_stream(s)
    bk.assert_quiescent()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        body()
    gr.replay()
    gr.replay()
    torch.cuda.synchronize()
    # eager + capture warm-up + 2 replays = 4 increments (the capture itself does not run the body)
    cap = {"cap_big": bool((g1 == 3).all()), "cap_small": bool((g2 == 6).all() and (g3 == 9).all()),
           "cap_zero": bool((full == 3).all())}
    fails += [k for k, v in cap.items() if not v]
    return fails


def runner(ws, graphs):
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.runner import Y2HRunner
    r = Y2HRunner()
    for k, v in dict(device="cuda", n_epochs=2, data_len=200, batch_size_DML=16, print_freq=1000, workspace=ws,
                     data_dir=os.path.join(ws, "nodata"), hip_graphs=graphs, seed=0).items():
        setattr(r, k, v)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        m = r.train_Conv_Linear_of_HDCE()
    torch.cuda.synchronize()
    return r, m


def main(out, ws):
    faulthandler.enable()
    ctx = init_distributed("cuda")
    fails = [] if (ctx.backend == "rccl" and ctx.distributed and ctx.comm is not None) else ["backend"]
    if not fails:
        fails += collectives(ctx)
        rg, mg = runner(os.path.join(ws, "g"), True)
        re_, me = runner(os.path.join(ws, "e"), False)
        same = torch.equal(mg.space.flat, me.space.flat) and all(
            torch.equal(a, b) for a, b in zip(mg.run_mean + mg.run_var, me.run_mean + me.run_var))
        if not (same and rg.train_HDCE_losses == re_.train_HDCE_losses and rg.val_HDCE_nmse == re_.val_HDCE_nmse):
            fails.append("runner_graphs_vs_eager")
    with open(f"{out}.{ctx.rank}", "w") as f:
        f.write(("1" if not fails else "0 " + ",".join(fails)) + "\n")
    shutdown()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
