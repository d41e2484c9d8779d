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


def test_hip_bn_recalibration_matches_torch(cuda):
    """Test-time BN re-estimation (Test.py's bn_adapt) on the HIP training conv forward == the torch
    (MIOpen) cumulative-average rule to bf16-conv accuracy; the expert with < 2 samples keeps its own
    statistics; restore_bn undoes both."""
    import copy
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.evaluate import recalibrate_bn, restore_bn
    convs, fc, _, _ = _models(cuda)
    ref_convs, hip_convs = copy.deepcopy(convs), copy.deepcopy(convs)
    eng = HIPInference(hip_convs, fc, 128, cuda, chunk=576)
    torch.manual_seed(1)
    N = 10003
    x = torch.randn(N, 2, 16, 8, device=cuda) * 0.7 + 0.1
    expert = torch.arange(N, device=cuda) % 2          # expert 2 gets nothing
    expert[:1] = 2                                     # ... one sample: < 2, skipped
    # (5001 samples per expert: chunks of 3000 + 2001 -- the last not a multiple of the BN tail's 8 samples per
    # workgroup, so its last workgroup is partial; rounds 3-4 refused such groups above 1365 samples, which broke
    # FIG1's bn_adapt sweep)
    saved_ref = recalibrate_bn(ref_convs, x, expert, chunk=3000)
    saved_hip = eng.recalibrate_bn(hip_convs, x, expert, chunk=3000)
    bn = lambda cs: [m for c in cs for m in c.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    for i, (a, b, o) in enumerate(zip(bn(ref_convs), bn(hip_convs), bn(convs))):
        e = i // 3
        if e == 2:
            assert torch.equal(b.running_mean, o.running_mean) and torch.equal(b.running_var, o.running_var)
            continue
        assert int(b.num_batches_tracked) == int(a.num_batches_tracked) >= 2
        s = a.running_var.sqrt().mean()
        assert torch.allclose(b.running_mean, a.running_mean, atol=0.02 * float(s), rtol=0.02), (i, float((b.running_mean - a.running_mean).abs().max()))
        assert torch.allclose(b.running_var, a.running_var, rtol=0.04, atol=1e-4), (i, float((b.running_var / a.running_var - 1).abs().max()))
    restore_bn(hip_convs, saved_hip)
    restore_bn(ref_convs, saved_ref)
    for a, o in zip(bn(hip_convs), bn(convs)):
        assert torch.equal(a.running_mean, o.running_mean) and torch.equal(a.running_var, o.running_var)
