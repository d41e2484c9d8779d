"""Hand-written MFMA FC GEMM (csrc/hip/fc_gemm.hip) vs an fp32 PyTorch reference: the plain bias
epilogue and the fused HDCE-loss epilogue (dY, loss, loss_perf, bias gradient, NaN flag)."""
import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import FcNmse, fc_linear, tile_m

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(288, 256, 320), (256, 384, 128), (2304, 2048, 4096)])
def test_fc_linear_matches_fp32(cuda, M, N, K):
    torch.manual_seed(0)
    A = torch.randn(M, K, device=cuda).bfloat16()
    W = (torch.randn(N, K, device=cuda) * K ** -0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    Y = fc_linear(A, W, b)
    ref = A.float() @ W.float().t() + b.float()
    torch.cuda.synchronize()
    assert tile_m(M, N, K) in (128, 144)
    err = (Y.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, float(err)
    # asymmetric check of the layout: one hot column of W
    W2 = torch.zeros(N, K, device=cuda, dtype=torch.bfloat16)
    W2[5, 7] = 1.0
    Y2 = fc_linear(A, W2, None)
    assert torch.equal(Y2[:, 5], A[:, 7]) and float(Y2[:, :5].abs().sum()) == 0.0


def _rows(E, U, B, N_store, cols, device):
    S = E * U
    L = torch.randn(S, N_store, cols, device=device)
    P = L + 0.3 * torch.randn_like(L)
    idx = torch.randint(0, N_store, (B,), device=device)
    u = torch.arange(U, device=device).view(U, 1, 1)
    e = torch.arange(E, device=device).view(1, 1, E)
    rowoff = ((e * U + u).expand(U, B, E) * N_store + idx.view(1, B, 1)).reshape(-1).to(torch.int32)
    lab = L.reshape(-1, cols)[rowoff.long()]
    per = P.reshape(-1, cols)[rowoff.long()]
    rowden = torch.stack([lab.pow(2).sum(1), per.pow(2).sum(1)], 1).contiguous()
    stream = (e * U + u).expand(U, B, E).reshape(-1)
    return L, P, rowoff, rowden, lab, per, stream


@pytest.mark.parametrize("E,U,B,N,K", [(3, 3, 32, 256, 320), (3, 3, 256, 2048, 4096)])
def test_fc_nmse_epilogue_matches_fp32(cuda, E, U, B, N, K):
    torch.manual_seed(1)
    M, S = E * U * B, E * U
    A = torch.randn(M, K, device=cuda).bfloat16()
    W = (torch.randn(N, K, device=cuda) * K ** -0.5).bfloat16()
    b = (0.1 * torch.randn(N, device=cuda)).bfloat16()
    L, P, rowoff, rowden, lab, per, stream = _rows(E, U, B, 40, N, cuda)
    op = FcNmse(M, N, K, (E, U, B), cuda)
    loss = torch.zeros(2, device=cuda)
    skip = torch.zeros(1, device=cuda)
    bg = torch.full((N,), 1e30, device=cuda)
    dY = op(A, W, b, L, P, rowoff, rowden, bg, loss, skip)
    torch.cuda.synchronize()
    Y = A.float() @ W.float().t() + b.float()
    num = torch.zeros(S, device=cuda).index_add_(0, stream, ((Y - lab) ** 2).sum(1))
    den = torch.zeros(S, device=cuda).index_add_(0, stream, (lab ** 2).sum(1))
    nump = torch.zeros(S, device=cuda).index_add_(0, stream, ((Y - per) ** 2).sum(1))
    denp = torch.zeros(S, device=cuda).index_add_(0, stream, (per ** 2).sum(1))
    ref_loss = torch.stack([(num / den).mean(), (nump / denp).mean()])
    coef = 2.0 / (S * den)
    ref_dY = coef[stream][:, None] * (Y - lab)
    assert torch.allclose(loss, ref_loss, rtol=2e-3), (loss, ref_loss)
    assert float((dY.float() - ref_dY).abs().max()) <= 2e-2 * float(ref_dY.abs().max())
    assert torch.allclose(bg, ref_dY.sum(0), rtol=2e-2, atol=2e-2 * float(ref_dY.sum(0).abs().max()))
    assert float(skip) == 0.0 and torch.allclose(op.ss[:, 1], den, rtol=1e-4)
    A[3, 3] = float("nan")
    op(A, W, b, L, P, rowoff, rowden, bg, loss, skip)
    torch.cuda.synchronize()
    assert float(skip) == 1.0
