"""Flagship step on the GPU: the fused kernels WRITE every gradient (no zero_grad needed)."""
import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import FlagshipConfig, FlagshipTrainer

pytestmark = pytest.mark.gpu


def _views(tr):
    out = []
    for sp in (tr.hdce.space, tr.qspace):
        out += [sp.grad[sp.slice_of(p)] for p in sp.params]
    return out


def test_no_zero_grad_overwrites_every_gradient(cuda):
    ctx = DistContext(device=cuda)
    cfg = FlagshipConfig(batch=32, data_len=400, hip_graphs=False, use_quantumnat=False)
    tr = FlagshipTrainer(cfg, ctx)
    tr.next_batch()
    # reference: zero_grad + accumulate
    tr.hstep.writes_grads, tr.cstep.writes_grads = False, False
    tr._phase1()
    tr._phase2()
    ref = [g.clone() for g in _views(tr)]
    # poison every parameter gradient, then the write-mode step must reproduce ref exactly
    for g in _views(tr):
        g.fill_(1e30)
    tr.hstep.writes_grads, tr.cstep.writes_grads = True, True
    tr._phase1()
    tr._phase2()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(_views(tr), ref)):
        assert torch.isfinite(a).all() and a.abs().max() < 1e29, i
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-7), (i, float((a - b).abs().max()))
