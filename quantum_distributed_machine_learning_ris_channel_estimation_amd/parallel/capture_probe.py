"""Pre-flight check: do RCCL collectives survive HIP graph capture on THIS node, at THIS world size?

The one-graph data-parallel plan (``FlagshipConfig.dp_one_graph``) captures the step's all-reduces
into its HIP graph.  That path is measured bit-exact over a one-rank RCCL group
(``tests/test_flagship_gpu.py::test_dp_one_graph_matches_five_graphs_over_rccl``), but a runtime that
cannot capture a collective fails hard (a segfault in ``hipStreamEndCapture`` was
seen with torch's process group in round 2), not with an exception.  So before a multi-rank run commits to it,
every rank starts a CHILD process (the parent has not touched the GPU yet) that captures the plan's
collective pattern through the framework's own RCCL communicator (``parallel/comm.py``) and
``GradBuckets`` -- two bucket all-reduces (one coalesced), one waited for on a forked stream, and the
ZeRO plan's reduce-scatter + all-gather -- replays it and checks the sums.  The
ranks then agree through a TCPStore: rank 0 publishes one decision (the plan is used only if every
child succeeded) and every rank reads it; a rank that cannot read it exits non-zero.

    ok = preflight(timeout=120)   # call before anything touches the GPU; True on every rank or none
"""
from __future__ import annotations

import datetime
import os
import subprocess
import sys
import time


def _child() -> int:
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import (GradBuckets,
                                                                                             init_distributed,
                                                                                             shutdown)
    ctx = init_distributed("cuda")
    rank, world, dev = ctx.rank, ctx.world, ctx.device
    a = torch.full((1 << 20,), float(rank + 1), device=dev)
    b = torch.full((4096,), 1.0, device=dev)
    c = torch.full((8,), 1.0, device=dev)
    out = torch.empty_like(a)
    # the ZeRO one-graph plan's collectives too: reduce-scatter of a region, all-gather of the shards
    full = torch.full((world * 8192,), float(rank + 1), device=dev)
    gath = torch.zeros(world * 8192, device=dev)
    bk = GradBuckets(ctx, {"a": [a], "bc": [b, c]})
    side = torch.cuda.Stream(dev)

    def body():
        a.mul_(1.0)
        bk.launch("a")
        bk.launch("bc", inline=True)   # (the DP step's small bucket: inline on the issuing stream)
        bk.launch_reduce_scatter("rs", full)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):   # (one bucket consumed on a forked stream)
            bk.wait(("a",))
            out.copy_(a)
        bk.wait(("bc", "rs"))
        gath.copy_(full)
        bk.launch_all_gather("ag", gath)
        bk.wait(("ag",))
        bk.clear()
        torch.cuda.current_stream(dev).wait_stream(side)

    def reset():
        a.fill_(float(rank + 1))
        b.fill_(1.0)
        c.fill_(1.0)
        full.fill_(float(rank + 1))
        gath.zero_()

    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    reset()
    with torch.cuda.graph(g):
        body()
    reset()
    g.replay()
    torch.cuda.synchronize(dev)
    tri = world * (world + 1) / 2
    ok = (bool((out == tri).all()) and bool((b == world).all()) and bool((c == world).all())
          and bool((gath.view(world, -1)[rank] == tri).all()))
    ctx.barrier()
    shutdown()
    return 0 if ok else 3


def preflight(timeout: float = 120.0, port_offset: int = 7) -> bool:
    """Run the capture probe in a child of every rank and agree on the result (see module docstring).
    Must be called before this process touches the GPU.  False on every rank if any rank's probe
    failed, crashed or timed out; SystemExit on a rank that cannot obtain the agreed decision."""
    import torch.distributed as dist
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    base = int(os.environ.get("MASTER_PORT", "29500"))
    env = dict(os.environ, MASTER_ADDR=host, MASTER_PORT=str(base + port_offset))
    # (under torchrun the env:// rendezvous would join the elastic agent's store at MASTER_PORT -- nobody
    # serves the probe's port: the child hosts its own store instead)
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    t0 = time.time()
    try:
        p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child"], env=env,
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=timeout, text=True)
        rc = p.returncode
        if rc != 0:
            tail = [ln for ln in p.stderr.splitlines() if ln.strip() and "Cannot find the function" not in ln][-6:]
            print(f"[capture preflight] rank {rank}: probe exit {rc}:\n  " + "\n  ".join(tail), file=sys.stderr, flush=True)
    except subprocess.TimeoutExpired:
        rc = 124
    # Agreement: every rank publishes its probe result; rank 0 alone decides and publishes ONE decision
    # key that every rank reads.  A rank that cannot take part (store unreachable, a read that fails
    # after the vote) exits non-zero instead of falling back to a default of its own: ranks running
    # different plans would issue different collective sequences (a hang or silent corruption).
    try:
        store = dist.TCPStore(host, base + port_offset + 1, world, rank == 0,
                              timeout=datetime.timedelta(seconds=timeout + 60))
        store.set(f"qdml_capture_ok_{rank}", "1" if rc == 0 else "0")
        if rank == 0:
            ok = all(store.get(f"qdml_capture_ok_{r}") == b"1" for r in range(world))
            store.set("qdml_capture_decision", "1" if ok else "0")
        ok = store.get("qdml_capture_decision") == b"1"
        store.set(f"qdml_capture_done_{rank}", "1")   # (rank 0 hosts the store: it must outlive every read)
        if rank == 0:
            for r in range(world):
                store.wait([f"qdml_capture_done_{r}"])
    except Exception as e:
        raise SystemExit(f"[capture preflight] rank {rank}: no agreed decision ({e}); exiting") from e
    if rank == 0:
        import torch
        print(f"[capture preflight] world {world}: {'ok' if ok else f'FAILED (rank 0 rc={rc})'} "
              f"in {time.time() - t0:.1f}s; devices visible after the probe: {torch._C._cuda_getDeviceCount()}",
              file=sys.stderr, flush=True)
    return ok


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.exit(_child())
