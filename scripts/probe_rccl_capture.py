"""Which RCCL collective patterns survive HIP graph capture (one GPU, an RCCL group of one rank)?

    python scripts/probe_rccl_capture.py            # runs every case in its own child process

Each case captures a small graph around torch.distributed collectives, replays it 3 times and
checks the result.  A case that crashes (segfault in hipStreamEndCapture) only ends its child."""
import os
import subprocess
import sys

CASES = ["ar_sync", "ar_async", "ar_async_side", "rs_async", "ag_async", "two_async", "two_streams"]


def case(name):
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29600 + CASES.index(name)))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    x = torch.ones(1 << 20, device="cuda")
    y = torch.empty(1 << 20, device="cuda")
    side = torch.cuda.Stream()

    def body():
        x.mul_(1.0)
        if name == "ar_sync":
            dist.all_reduce(x)
        elif name == "ar_async":
            dist.all_reduce(x, async_op=True).wait()
        elif name == "ar_async_side":
            w = dist.all_reduce(x, async_op=True)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w.wait()
                y.copy_(x)
            torch.cuda.current_stream().wait_stream(side)
        elif name == "rs_async":
            dist.reduce_scatter_tensor(y, x, async_op=True).wait()
        elif name == "ag_async":
            dist.all_gather_into_tensor(y, x, async_op=True).wait()
        elif name == "two_async":
            w1 = dist.all_reduce(x, async_op=True)
            w2 = dist.all_reduce(y, async_op=True)
            w1.wait()
            w2.wait()
        elif name == "two_streams":   # the DP plan's shape: a collective launched from a side stream
            w1 = dist.reduce_scatter_tensor(y, x, async_op=True)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w1.wait()
                w2 = dist.all_gather_into_tensor(x, y, async_op=True)
                w2.wait()
            torch.cuda.current_stream().wait_stream(side)
        y.add_(1.0)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for mode in ("thread_local", "relaxed", "global"):
        g = torch.cuda.CUDAGraph()
        print(f"{name}: capturing ({mode})", flush=True)
        with torch.cuda.graph(g, capture_error_mode=mode):
            body()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        print(f"{name}: OK ({mode})", flush=True)
        break
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 1:
        case(sys.argv[1])
        return 0
    for c in CASES:
        p = subprocess.run([sys.executable, "-u", __file__, c], capture_output=True, text=True, timeout=120)
        lines = [ln for ln in (p.stdout + p.stderr).splitlines() if c in ln or "Error" in ln][-3:]
        print(f"{c:14s} rc={p.returncode}  " + " | ".join(lines), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
