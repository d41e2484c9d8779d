"""Run under the launcher (world 2, gloo): DP over per-rank batches == 1 process on the union."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import SC_P128  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.optim import (  # noqa: E402
    FlatParamSpace, FusedOptimizer)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import (  # noqa: E402
    DeviceSampler, GradBuckets, init_distributed, shutdown)


def build():
    torch.manual_seed(0)
    m = SC_P128()
    space = FlatParamSpace(list(m.named_parameters()))
    return m, space, FusedOptimizer(space, "adam", 1e-2)


def main():
    out = sys.argv[1]
    ctx = init_distributed("cpu")
    assert ctx.world == 2 and ctx.backend == "gloo"
    torch.manual_seed(123)
    X = torch.randn(16, 2, 16, 8)
    Y = torch.randint(0, 3, (16,))
    m, space, opt = build()
    # rank-0 broadcast of initial weights (ranks could differ otherwise)
    if ctx.rank == 1:
        with torch.no_grad():
            space.flat.add_(1.0)
    ctx.broadcast_(space.flat)
    # two buckets, one coalesced from two tensors
    n0 = space.offsets[2]
    buckets = GradBuckets(ctx, {"a": [space.grad[:n0]], "b": [space.grad[n0:n0 + 100], space.grad[n0 + 100:]]})
    for step in range(3):
        sl = slice(ctx.rank * 8, (ctx.rank + 1) * 8)
        space.zero_grad()
        F.nll_loss(m(X[sl]), Y[sl]).backward()
        buckets.launch_all()
        buckets.wait()
        opt.step(grad_scale=1.0 / ctx.world)
    # single-process reference on the union batch
    m1, s1, o1 = build()
    for step in range(3):
        s1.zero_grad()
        F.nll_loss(m1(X), Y).backward()
        o1.step()
    err = float((space.flat - s1.flat).abs().max())
    # global metric reduction: sums, not mean of ratios
    num = torch.tensor([1.0 + ctx.rank, 10.0 * (1 + 3 * ctx.rank)])
    ctx.all_reduce_(num)
    # sampler shards are disjoint per rank seed
    idx = next(iter(DeviceSampler(100, 10, "cpu", seed=0, rank=ctx.rank)))
    with open(f"{out}.{ctx.rank}", "w") as f:
        f.write(f"{err} {num[0].item()} {num[1].item()} {idx.tolist()}\n")
    shutdown()


if __name__ == "__main__":
    main()
