"""Fused HIP QSC step (csrc/hip/qsc.hip + qsim.hip) vs torch autograd of the same QSC_P128."""
import pytest
import torch
import torch.nn.functional as F

from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import QSC_P128
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.optim import FlatParamSpace
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.qsc import QSCStepHIP

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pilot_num,n,B", [(128, 8, 2304), (128, 4, 300), (128, 6, 64), (256, 6, 96),
                                                   (256, 12, 72), (128, 16, 18)])
def test_qsc_step_matches_autograd(cuda, pilot_num, n, B):
    torch.manual_seed(0)
    H, W = (16, 8) if pilot_num == 128 else (16, 16)
    a = QSC_P128(n_qubits=n, use_quantumnat=False, use_gradient_pruning=False, pilot_num=pilot_num).to(cuda)
    b = QSC_P128(n_qubits=n, use_quantumnat=False, use_gradient_pruning=False, pilot_num=pilot_num).to(cuda)
    b.load_state_dict(a.state_dict())
    space = FlatParamSpace(list(a.named_parameters()), cuda)
    x = torch.randn(B, 2, H, W, device=cuda)
    y = torch.randint(0, 3, (B,), device=cuda)
    step = QSCStepHIP(a, space, B)
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
