"""Debug: gloo collectives on CUDA tensors, 2 ranks sharing one GPU (QDML_DIST_BACKEND=gloo)."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import init_distributed  # noqa: E402

ctx = init_distributed("cuda")
r = ctx.rank
t = torch.full((4,), float(r + 1), device=ctx.device)
v = t[1:2]
w = dist.all_reduce(v, async_op=True)
w.wait()
torch.cuda.synchronize()
print(r, "view allreduce", t.tolist(), flush=True)
s = torch.cuda.Stream()
x = torch.full((1000,), float(r + 1), device=ctx.device)
x.mul_(2)   # queued work before the collective
w = dist.all_reduce(x, async_op=True)
with torch.cuda.stream(s):
    w.wait()
    y = x * 1.0
torch.cuda.synchronize()
print(r, "side-stream wait", float(x[0]), float(y[0]), flush=True)
dist.destroy_process_group()
