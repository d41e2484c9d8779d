"""Fused HIP QSC step (csrc/hip/qsc.hip + qsim.hip) vs torch autograd of the same QSC_P128."""
import pytest
import torch
import torch.nn.functional as F

from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import QSC_P128
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.optim import FlatParamSpace
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.qsc import QSCStepHIP

from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("impl", ["mfma", "ref"])
@pytest.mark.parametrize("pilot_num,n,B", [(128, 8, 2304), (128, 4, 300), (128, 6, 64), (256, 6, 96),
                                                   (256, 12, 72), (128, 16, 18)])
def test_qsc_step_matches_autograd(cuda, pilot_num, n, B, impl):
    torch.manual_seed(0)
    H, W = (16, 8) if pilot_num == 128 else (16, 16)
    a = QSC_P128(n_qubits=n, use_quantumnat=False, use_gradient_pruning=False, pilot_num=pilot_num).to(cuda)
    b = QSC_P128(n_qubits=n, use_quantumnat=False, use_gradient_pruning=False, pilot_num=pilot_num).to(cuda)
    b.load_state_dict(a.state_dict())
    space = FlatParamSpace(list(a.named_parameters()), cuda)
    x = torch.randn(B, 2, H, W, device=cuda)
    y = torch.randint(0, 3, (B,), device=cuda)
    step = QSCStepHIP(a, space, B, impl=impl)
    space.zero_grad()
    loss = step(x, y)
    ref = F.nll_loss(b(x), y)
    ref.backward()
    torch.cuda.synchronize()
    assert torch.allclose(loss[0], ref, rtol=1e-4, atol=1e-5), (loss, ref)
    for (na, pa), (nb, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert na == nb
        err = (pa.grad - pb.grad).abs().max() / pb.grad.abs().max().clamp_min(1e-12)
        assert err < 2e-3, (na, float(err))


def test_qsc_step_quantumnat_in_kernel_noise(cuda):
    """QuantumNAT noise drawn in-kernel: N(0, sigma^2) per element, fresh every step, distinct per
    stream group; the fused step equals autograd through the SAME noisy weights, grads to the master."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.quantum import qsim
    torch.manual_seed(0)
    n, G, b = 6, 9, 32
    B = G * b
    a = QSC_P128(n_qubits=n, use_quantumnat=True, use_gradient_pruning=False, noise_level=0.05).to(cuda)
    ref = QSC_P128(n_qubits=n, use_quantumnat=False, use_gradient_pruning=False).to(cuda)
    ref.load_state_dict(a.state_dict())
    space = FlatParamSpace(list(a.named_parameters()), cuda)
    step = QSCStepHIP(a, space, B, n_groups=G)
    x = torch.randn(B, 2, 16, 8, device=cuda)
    y = torch.randint(0, 3, (B,), device=cuda)
    space.zero_grad()
    loss = step(x, y)
    wn = step.wnoisy.clone()
    w0 = a.qlayer.weights.detach()
    d = (wn - w0.unsqueeze(0)) / 0.05
    assert abs(float(d.mean())) < 0.1 and abs(float(d.std()) - 1.0) < 0.1
    assert not torch.equal(wn[0], wn[1])
    # reference through the same noisy weights
    angles = ref.preprocess(x)
    wq = ref.qlayer.weights.unsqueeze(0) + (wn - w0.unsqueeze(0))
    out = F.log_softmax(ref.classifier(qsim(angles, wq, "hip")), dim=1)
    rl = F.nll_loss(out, y)
    rl.backward()
    torch.cuda.synchronize()
    assert torch.allclose(loss[0], rl, rtol=1e-4, atol=1e-5)
    for (na, pa), (nb, pb) in zip(a.named_parameters(), ref.named_parameters()):
        err = (pa.grad - pb.grad).abs().max() / pb.grad.abs().max().clamp_min(1e-12)
        assert err < 2e-3, (na, float(err))
    # next step: fresh noise
    step(x, y)
    assert not torch.equal(step.wnoisy, wn)


@pytest.mark.parametrize("n,B", [(8, 2304), (4, 300), (16, 18)])
def test_qsc_bwd_bf16x3_matches_f32_kernel(cuda, n, B):
    """P128 backward on bf16x3 MFMAs (qsc2_bwd3_kernel: hi/lo bf16 operands, three products) vs the
    f32-MFMA kernel on the same forward: fp32-grade agreement on every parameter gradient."""
    torch.manual_seed(0)
    a = QSC_P128(n_qubits=n, use_quantumnat=False, use_gradient_pruning=False).to(cuda)
    space = FlatParamSpace(list(a.named_parameters()), cuda)
    x = torch.randn(B, 2, 16, 8, device=cuda)
    y = torch.randint(0, 3, (B,), device=cuda)
    step = QSCStepHIP(a, space, B)
    assert step.bwd_x3
    out = []
    for x3 in (True, False):
        step.bwd_x3 = x3
        space.zero_grad()
        loss = step(x, y).clone()
        torch.cuda.synchronize()
        out.append((loss, {k: p.grad.clone() for k, p in a.named_parameters()}))
    (l3, g3), (l32, g32) = out
    assert torch.equal(l3, l32)
    # forward: conv2 on bf16x3 (qd_qsc2_fwd3) vs f32 MFMAs -- the angles the circuit consumes
    angles = []
    for x3 in (True, False):
        step.fwd_x3 = x3
        step(x, y)
        torch.cuda.synchronize()
        angles.append(step.angles.clone())
    err = float((angles[0] - angles[1]).abs().max() / angles[1].abs().max())
    print(f"angles: bf16x3 vs f32 forward max-rel {err:.2e}")
    assert err < 1e-4, err
    for k in g32:
        err = float((g3[k] - g32[k]).abs().max() / g32[k].abs().max().clamp_min(1e-12))
        print(f"{k}: bf16x3 vs f32 max-rel {err:.2e}")
        assert err < 1e-4, (k, err)


@pytest.mark.parametrize("noise", [False, True])
def test_qsc_circuit_forward_on_mfma_matches_register_kernel(cuda, monkeypatch, noise):
    """The flagship's 8-qubit circuit forward on the matrix cores (qsim_mfma.hip, operand images built in the
    QuantumNAT draw's launch) == the register kernel (qsim.hip): the same noisy weights bit for bit, the same
    draw counter, <Z> / loss / every gradient to fp32 accuracy, over two steps."""
    G, B = 9, 2304
    outs = []
    for mf in ("1", "0"):
        monkeypatch.setattr(KNOBS, "qsim_mfma", mf == "1")
        torch.manual_seed(0)
        a = QSC_P128(n_qubits=8, use_quantumnat=noise, use_gradient_pruning=False, pilot_num=128).to(cuda)
        a.train()
        space = FlatParamSpace(list(a.named_parameters()), cuda)
        torch.manual_seed(1)
        step = QSCStepHIP(a, space, B, n_groups=G)
        assert step.mfma == (mf == "1")
        x = torch.randn(B, 2, 16, 8, device=cuda)
        y = torch.randint(0, 3, (B,), device=cuda)
        rec = []
        for _ in range(2):
            space.zero_grad()
            loss = step(x, y)
            torch.cuda.synchronize()
            rec.append((loss.clone(), step.E.clone(), space.grad.clone(), step.wnoisy.clone(), step.noise_ctr.clone()))
        outs.append(rec)
    for (la, ea, ga, wa, ca), (lb, eb, gb, wb, cb) in zip(*outs):
        if noise:
            assert torch.equal(wa, wb) and torch.equal(ca, cb)
        assert torch.allclose(la, lb, rtol=1e-5, atol=1e-6), (la, lb)
        assert float((ea - eb).abs().max()) < 2e-5
        assert float((ga - gb).abs().max()) <= 1e-4 * float(gb.abs().max())


@pytest.mark.parametrize("n", [4, 8])
def test_classifier_validation_runs_on_hip_kernels(cuda, n):
    """The runner's QSC validation (ClassifierStep.forward in eval mode) runs the HIP inference kernels
    (QSCStepHIP.infer: preprocess CNN, circuit on the clean weights, inference head) in chunks of the static
    batch -- the last one padded -- and matches the models' torch forward (reference R:378-414)."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import ClassifierStep
    torch.manual_seed(3)
    m = QSC_P128(n_qubits=n, use_quantumnat=True, use_gradient_pruning=False, pilot_num=128).to(cuda)
    space = FlatParamSpace(list(m.named_parameters()), cuda)
    cs = ClassifierStep(m, 9, space=space, batch_total=9 * 32)
    assert cs.hip is not None and cs.hip.impl == "mfma"
    x = torch.randn(9 * 32 * 2 + 50, 2, 16, 8, device=cuda)      # two full chunks + a partial one
    m.eval()
    got = cs.forward(x)
    ref = F.log_softmax(m.classifier(m.qlayer(m.preprocess(x))), dim=1)
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    assert float((got - ref).abs().max()) < 2e-4, float((got - ref).abs().max())
    assert torch.equal(got.argmax(1), ref.argmax(1))


def test_qsc_fwd_conv1_on_mfma_matches_f32_forward(cuda):
    """Round 6: the P128 forward's conv1 + ReLU + pool 1 on f32 MFMAs (qsc_mfma.hip conv1_mfma, the bf16x3 forward)
    vs the f32 forward's VALU conv1: the saved pool-1 map agrees to fp32 grade and the saved window choices (2-bit
    codes per channel) everywhere but near-ties."""
    torch.manual_seed(1)
    B = 2304
    a = QSC_P128(n_qubits=8, use_quantumnat=False, use_gradient_pruning=False).to(cuda)
    space = FlatParamSpace(list(a.named_parameters()), cuda)
    x = torch.randn(B, 2, 16, 8, device=cuda)
    y = torch.randint(0, 3, (B,), device=cuda)
    step = QSCStepHIP(a, space, B)
    assert step.fwd_x3
    saved = []
    for x3 in (True, False):
        step.fwd_x3 = x3
        step.forward_part(x, y)
        torch.cuda.synchronize()
        saved.append((step.p1s.clone(), step.c1.clone(), step.angles.clone()))
    (p3, c3, a3), (pf, cf, af) = saved
    shifts = torch.arange(0, 32, 2, device=cuda, dtype=torch.int32)
    k3 = (c3.unsqueeze(-1) >> shifts) & 3
    kf = (cf.unsqueeze(-1) >> shifts) & 3
    diff = float((k3 != kf).float().mean())
    err = float((p3 - pf).abs().max() / pf.abs().max())
    print(f"conv1 MFMA vs f32: window-choice mismatch {diff:.2e}, pool-1 max-rel {err:.2e}")
    assert diff < 1e-4, diff
    assert err < 1e-5, err
    assert float((a3 - af).abs().max()) < 1e-4


@pytest.mark.parametrize("pilot", [128, 256])
def test_qsc_pool1_map_and_choices_match_torch(cuda, pilot):
    """Round 6: the QSC forward's conv1 + ReLU + pool 1 on f32 MFMAs (P128: conv1_mfma, P256: conv1_mfma16) against
    torch's conv2d / relu / max_pool2d on the same input: the saved pool-1 map (the backward's ReLU mask) to fp32
    grade and the saved window choices (2-bit codes, first max in scan order) equal to max_pool2d's indices but for
    near-ties."""
    import torch.nn.functional as F
    torch.manual_seed(3)
    B = 288
    H, W = (16, 8) if pilot == 128 else (16, 16)
    m = QSC_P128(n_qubits=8, use_quantumnat=False, use_gradient_pruning=False, pilot_num=pilot).to(cuda)
    space = FlatParamSpace(list(m.named_parameters()), cuda)
    x = torch.randn(B, 2, H, W, device=cuda)
    y = torch.randint(0, 3, (B,), device=cuda)
    step = QSCStepHIP(m, space, B)
    step.forward_part(x, y)
    torch.cuda.synchronize()
    conv = m.preprocess[0]
    with torch.no_grad():
        z = F.relu(F.conv2d(x, conv.weight, conv.bias, padding=1))
        pooled, idx = F.max_pool2d(z, 2, return_indices=True)          # (B, 16, H/2, W/2)
    ref = pooled.permute(0, 2, 3, 1).reshape(B, -1)                     # [window][channel]
    err = float((step.p1s - ref).abs().max() / ref.abs().max())
    qy = torch.arange(H // 2, device=cuda).view(1, 1, -1, 1)
    qx = torch.arange(W // 2, device=cuda).view(1, 1, 1, -1)
    code_ref = 2 * (idx // W - 2 * qy) + (idx % W - 2 * qx)            # 0 TL, 1 TR, 2 BL, 3 BR
    code_ref = code_ref.permute(0, 2, 3, 1).reshape(B, -1, 16)          # [sample][window][channel]
    shifts = torch.arange(0, 32, 2, device=cuda, dtype=torch.int32)
    code = (step.c1.unsqueeze(-1) >> shifts) & 3
    diff = float((code != code_ref).float().mean())
    print(f"P{pilot} pool-1 vs torch: max-rel {err:.2e}, window-choice mismatch {diff:.2e}")
    assert err < 1e-5, err
    assert diff < 1e-3, diff
