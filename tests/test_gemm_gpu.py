"""Hand-written FC GEMMs (csrc/hip/gemm.hip) vs an fp32 PyTorch reference: forward (KC x KC), weight
gradient (MC x MC, fp32 out) and data gradient (KC x MC), every tile configuration, with exact
one-hot checks of the layouts (an asymmetric operand catches any transposed / swapped indexing)."""
import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import (gemm_dgrad, gemm_fwd,
                                                                                  gemm_fwd_ok, gemm_wgrad)

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("cfg", [0, 1])
@pytest.mark.parametrize("M,N,K", [(576, 256, 192), (2304, 2048, 4096)])
def test_gemm_fwd_matches_fp32(cuda, cfg, M, N, K):
    if not gemm_fwd_ok(M, N, K, cfg):
        pytest.skip("shape not tiled by this cfg")
    torch.manual_seed(0)
    A = torch.randn(M, K, device=cuda).bfloat16()
    W = (torch.randn(N, K, device=cuda) * K ** -0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    Y = gemm_fwd(A, W, b, cfg=cfg)
    ref = A.float() @ W.float().t() + b.float()
    torch.cuda.synchronize()
    assert _rel(Y, ref) < 1e-2
    W2 = torch.zeros(N, K, device=cuda, dtype=torch.bfloat16)
    W2[5, 7] = 1.0
    W2[N - 3, K - 1] = 2.0
    Y2 = gemm_fwd(A, W2, None, cfg=cfg)
    torch.cuda.synchronize()
    assert torch.equal(Y2[:, 5], A[:, 7]) and torch.equal(Y2[:, N - 3], 2 * A[:, K - 1])
    assert float(Y2[:, :5].abs().sum()) == 0.0


@pytest.mark.parametrize("cfg", [0, 1])
@pytest.mark.parametrize("M,N,K", [(192, 256, 512), (2304, 2048, 4096)])
def test_gemm_wgrad_matches_fp32(cuda, cfg, M, N, K):
    torch.manual_seed(1)
    dY = (torch.randn(M, N, device=cuda) * 1e-2).bfloat16()
    A = torch.randn(M, K, device=cuda).bfloat16()
    dW = torch.full((N, K), 1e30, device=cuda)
    gemm_wgrad(dY, A, out=dW, cfg=cfg)
    ref = dY.float().t() @ A.float()
    torch.cuda.synchronize()
    assert _rel(dW, ref) < 1e-4   # fp32 accumulation of bf16 products: only summation order differs
    # layout: one hot row of dY / column of A
    dY2 = torch.zeros(M, N, device=cuda, dtype=torch.bfloat16)
    dY2[M - 1, 3] = 1.0
    dY2[2, N - 1] = -1.0
    dW2 = gemm_wgrad(dY2, A, cfg=cfg)
    torch.cuda.synchronize()
    assert torch.equal(dW2[3], A[M - 1].float()) and torch.equal(dW2[N - 1], -A[2].float())
    assert float(dW2[4:N - 1].abs().sum()) == 0.0


@pytest.mark.parametrize("cfg", [0, 1])
@pytest.mark.parametrize("M,N,K", [(288, 192, 256), (2304, 2048, 4096)])
def test_gemm_dgrad_matches_fp32(cuda, cfg, M, N, K):
    if cfg == 0 and K % 256:
        pytest.skip("cfg 0 tiles K by 256")
    torch.manual_seed(2)
    dY = (torch.randn(M, N, device=cuda) * 1e-2).bfloat16()
    W = (torch.randn(N, K, device=cuda) * N ** -0.5).bfloat16()
    dA = gemm_dgrad(dY, W, cfg=cfg)
    ref = dY.float() @ W.float()
    torch.cuda.synchronize()
    assert _rel(dA, ref) < 1e-2
    W2 = torch.zeros(N, K, device=cuda, dtype=torch.bfloat16)
    W2[N - 1, 5] = 1.0
    W2[0, K - 1] = 1.0
    dA2 = gemm_dgrad(dY, W2, cfg=cfg)
    torch.cuda.synchronize()
    assert torch.equal(dA2[:, 5], dY[:, N - 1]) and torch.equal(dA2[:, K - 1], dY[:, 0])
    assert float(dA2[:, :5].abs().sum()) == 0.0
