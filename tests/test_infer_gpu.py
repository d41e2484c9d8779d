"""Test-time hierarchical estimation on the HIP kernels (train/infer.py) vs the PyTorch routed path:
classifier predictions (SC_P128 exactly, QSC_P128 up to near-ties), and the routed estimate (every
sample through its predicted expert + the shared FC, routing fused into the GEMM) to bf16 accuracy."""
import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import (Conv_P128, FC_P128,
                                                                                             QSC_P128, SC_P128)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import estimate_routed
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.infer import HIPInference

pytestmark = pytest.mark.gpu


def _models(dev):
    torch.manual_seed(0)
    convs = [Conv_P128(128).to(dev).eval() for _ in range(3)]
    for c in convs:   # non-trivial running statistics
        for mod in c.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.2, 0.2)
                mod.running_var.uniform_(0.5, 2.0)
                mod.weight.data.uniform_(0.5, 1.5)
                mod.bias.data.uniform_(-0.1, 0.1)
    fc = FC_P128(128).to(dev).eval()
    sc = SC_P128(128).to(dev).eval()
    qsc = QSC_P128(8, 3, 3, False, False, 128).to(dev).eval()
    return convs, fc, sc, qsc


def test_hip_inference_matches_torch_routing(cuda):
    convs, fc, sc, qsc = _models(cuda)
    eng = HIPInference(convs, fc, 128, cuda, chunk=576, sc=sc, qsc=qsc)
    N = 1500   # (not a multiple of the chunk: the tail is padded)
    x = torch.randn(N, 2, 16, 8, device=cuda)
    with torch.no_grad():
        ref_sc = sc(x).argmax(1)
        ref_q = qsc(x).argmax(1)
    p_sc = eng.classify(x, "classical")
    p_q = eng.classify(x, "quantum")
    torch.cuda.synchronize()
    assert torch.equal(p_sc, ref_sc)
    assert float((p_q != ref_q).float().mean()) < 5e-3
    expert = torch.randint(0, 3, (N,), device=cuda)
    H = eng.estimate(x, expert)
    ref = estimate_routed(convs, fc, x, expert)
    torch.cuda.synchronize()
    err = float((H - ref).norm() / ref.norm())
    assert err < 1e-2, err
    # routing really selects per sample: a permuted expert vector changes exactly those rows
    e2 = (expert + 1) % 3
    H2 = eng.estimate(x, e2)
    torch.cuda.synchronize()
    assert float((H2 - estimate_routed(convs, fc, x, e2)).norm() / ref.norm()) < 1e-2
