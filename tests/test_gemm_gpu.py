"""Hand-written FC GEMMs (csrc/hip/gemm.hip) vs an fp32 PyTorch reference: forward (KC x KC), weight
gradient (MC x MC, fp32 out) and data gradient (KC x MC), every tile configuration, with exact
one-hot checks of the layouts (an asymmetric operand catches any transposed / swapped indexing)."""
import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import (gemm_dgrad, gemm_fwd,
                                                                                  gemm_fwd_ok, gemm_wgrad)

from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS
pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10])
@pytest.mark.parametrize("M,N,K", [(576, 256, 192), (576, 256, 256), (2304, 2048, 4096)])
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


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("M,N,K", [(192, 256, 512), (256, 256, 512), (2304, 2048, 4096)])
def test_gemm_wgrad_matches_fp32(cuda, cfg, M, N, K):
    if cfg == 2 and M % 128:
        pytest.skip("cfg 2 (K split over two wave groups) runs the M reduction in pairs of 64")
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


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("M,N,K", [(288, 192, 256), (288, 256, 256), (2304, 2048, 4096)])
def test_gemm_dgrad_matches_fp32(cuda, cfg, M, N, K):
    if cfg in (0, 2, 3) and K % 256:
        pytest.skip("cfg 0 / 2 / 3 tile K by 256")
    if cfg == 3 and N % 128:
        pytest.skip("cfg 3 (K split over two wave groups) runs the N reduction in pairs of 64")
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


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 5, 6, 7, 8, 10])
@pytest.mark.parametrize("E,U,B,N,K", [(3, 3, 64, 256, 320), (3, 3, 64, 256, 384), (3, 3, 256, 2048, 4096)])
def test_gemm_nmse_epilogue_matches_fp32(cuda, cfg, E, U, B, N, K):
    """Forward GEMM with the HDCE loss epilogue + finish: loss, loss_perf, dY, bias gradient, NaN flag."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import gemm_tile_m
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.nmse import StreamNMSE
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel
    torch.manual_seed(1)
    M, S = E * U * B, E * U
    if M % gemm_tile_m(cfg) or not gemm_fwd_ok(M, N, K, cfg):
        pytest.skip("shape not tiled by this cfg")
    A = torch.randn(M, K, device=cuda).bfloat16()
    W = (torch.randn(N, K, device=cuda) * K ** -0.5).bfloat16()
    b = (0.1 * torch.randn(N, device=cuda)).bfloat16()
    L, P, rowoff, rowden, lab, per, stream = _rows(E, U, B, 40, N, cuda)
    nm = StreamNMSE(HDCEModel.row_stream(E, U, B, cuda), S, N)
    nm.rowoff = rowoff
    bg = torch.full((N,), 1e30, device=cuda)
    dY = nm.gemm_fused(A, W, b, L, P, bg, (E, U, B), rowden, cfg=cfg)
    torch.cuda.synchronize()
    Y = A.float() @ W.float().t() + b.float()
    num = torch.zeros(S, device=cuda).index_add_(0, stream, ((Y - lab) ** 2).sum(1))
    den = torch.zeros(S, device=cuda).index_add_(0, stream, (lab ** 2).sum(1))
    nump = torch.zeros(S, device=cuda).index_add_(0, stream, ((Y - per) ** 2).sum(1))
    denp = torch.zeros(S, device=cuda).index_add_(0, stream, (per ** 2).sum(1))
    ref_loss = torch.stack([(num / den).mean(), (nump / denp).mean()])
    ref_dY = (2.0 / (S * den))[stream][:, None] * (Y - lab)
    assert torch.allclose(nm.loss, ref_loss, rtol=2e-3), (nm.loss, ref_loss)
    assert _rel(dY, ref_dY) <= 2e-2
    assert torch.allclose(bg, ref_dY.sum(0), rtol=2e-2, atol=2e-2 * float(ref_dY.sum(0).abs().max()))
    assert float(nm.skip) == 0.0 and torch.allclose(nm.ss[:, 1], den, rtol=1e-4)
    A[3, 3] = float("nan")
    nm.gemm_fused(A, W, b, L, P, bg, (E, U, B), rowden, cfg=cfg)
    torch.cuda.synchronize()
    assert float(nm.skip) == 1.0


def test_flagship_hand_gemm_matches_hipblaslt_path(cuda, monkeypatch):
    """One flagship step with the hand-written FC GEMMs (loss fused into the forward's epilogue) vs the
    hipBLASLt + one-pass NMSE path: loss and every gradient agree to bf16 accuracy."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (FlagshipConfig,
                                                                                                FlagshipTrainer)
    ctx = DistContext(device=cuda)
    cfg = dict(batch=64, data_len=800, hip_graphs=False, use_quantumnat=False, stream_mode="serial")
    trs = []
    for hand in ("1", "0"):
        monkeypatch.setattr(KNOBS, "hand_gemm", hand)
        tr = FlagshipTrainer(FlagshipConfig(**cfg), ctx)
        assert bool(tr.hstep.hand_gemm) == (hand == "1")
        tr.next_batch()
        tr._dp_g1()
        tr._dp_g2()
        torch.cuda.synchronize()
        trs.append(tr)
    a, b = trs
    assert torch.allclose(a.hloss, b.hloss, rtol=1e-2), (a.hloss, b.hloss)
    ga, gb = a.hdce.space.grad, b.hdce.space.grad
    sp = a.hdce.space
    for name, p in zip(sp.names, sp.params):
        sl = sp.slice_of(p)
        x, y = ga[sl], gb[sl]
        assert float((x - y).abs().max()) <= 3e-2 * float(y.abs().max()) + 1e-8, name


@pytest.mark.parametrize("cfg", ["2,1,2", None])
def test_flagship_plain_hand_forward_matches_library_forward(cuda, monkeypatch, cfg):
    """The hand-written FC forward with only the bias in its epilogue (KNOBS.hand_gemm "fwdplain": the loss as the
    separate one-pass NMSE kernel, as after hipBLASLt) vs the hipBLASLt forward: one flagship step, loss and
    every HDCE gradient to bf16 accuracy."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (FlagshipConfig,
                                                                                                FlagshipTrainer)
    ctx = DistContext(device=cuda)
    if cfg is not None:
        monkeypatch.setattr(KNOBS, "gemm_cfg", cfg)
    trs = []
    # (hg None: the defaults -- the shipped step runs this forward)
    for hg, path in ((None if cfg is None else "fwdplain,wgrad,dgrad", "hand_plain"), ("wgrad,dgrad", "library")):
        monkeypatch.setattr(KNOBS, "hand_gemm", "fwdplain,wgrad,dgrad" if hg is None else hg)
        torch.manual_seed(0)
        tr = FlagshipTrainer(FlagshipConfig(batch=192, data_len=800, hip_graphs=False, use_quantumnat=False,
                                            stream_mode="serial"), ctx)
        tr.next_batch()
        tr._dp_g1()
        tr._dp_g2()
        torch.cuda.synchronize()
        assert tr.hstep.fc_path == path
        trs.append(tr)
    a, b = trs
    assert torch.allclose(a.hloss, b.hloss, rtol=1e-2), (a.hloss, b.hloss)
    sp = a.hdce.space
    for name, p in zip(sp.names, sp.params):
        sl = sp.slice_of(p)
        x, y = a.hdce.space.grad[sl], b.hdce.space.grad[sl]
        assert float((x - y).abs().max()) <= 3e-2 * float(y.abs().max()) + 1e-8, name


@pytest.mark.parametrize("cfg", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(576, 256, 256), (2304, 2048, 4096)])
def test_gemm_fwd_f8_matches_fp32(cuda, M, N, K, cfg):
    """e4m3 forward (mfma_f32_16x16x32_fp8_fp8, two per 16-byte fragment) == the fp32 product of the SAME
    dequantised operands (the only error left is fp32 accumulation order + the bf16 output), and exact
    one-hot layout checks."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import gemm_fwd_f8
    torch.manual_seed(2)
    A = torch.randn(M, K, device=cuda)
    W = torch.randn(N, K, device=cuda) * K ** -0.5
    sa, sw = float(A.abs().max()) / 448.0, float(W.abs().max()) / 448.0
    A8 = (A / sa).to(torch.float8_e4m3fn)
    W8 = (W / sw).to(torch.float8_e4m3fn)
    deq = torch.tensor([sa, sw], device=cuda)
    b = torch.randn(N, device=cuda).bfloat16()
    Y = gemm_fwd_f8(A8, W8, deq, b, cfg=cfg)
    ref = (A8.float() * sa) @ (W8.float() * sw).t() + b.float()
    torch.cuda.synchronize()
    assert _rel(Y, ref) < 8e-3, _rel(Y, ref)
    W2 = torch.zeros(N, K, device=cuda)
    W2[5, 7] = 1.0
    W2[N - 3, K - 1] = 2.0
    Y2 = gemm_fwd_f8(A8, W2.to(torch.float8_e4m3fn), torch.tensor([1.0, 1.0], device=cuda), cfg=cfg)
    torch.cuda.synchronize()
    assert torch.equal(Y2[:, 5].float(), A8[:, 7].float().bfloat16().float())
    assert torch.equal(Y2[:, N - 3].float(), (2 * A8[:, K - 1].float()).bfloat16().float())
    assert float(Y2[:, :5].float().abs().sum()) == 0.0


def test_flagship_fp8_hand_gemm_matches_scaled_mm_path(cuda, monkeypatch):
    """fp8 estimator step: the hand-written e4m3 GEMM with the loss epilogue vs hipBLASLt's scaled GEMM +
    the one-pass NMSE kernel, from the same e4m3 operands and scales: loss and every gradient agree."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (FlagshipConfig,
                                                                                                FlagshipTrainer)
    ctx = DistContext(device=cuda)
    cfg = dict(batch=64, data_len=800, hip_graphs=False, use_quantumnat=False, stream_mode="serial", dtype="fp8")
    trs = []
    monkeypatch.setattr(KNOBS, "f8_bwd", False)   # (bf16 gradients on both sides; the e4m3 backward: next test)
    for hand in ("1", "0"):
        monkeypatch.setattr(KNOBS, "hand_fp8", hand == "1")
        tr = FlagshipTrainer(FlagshipConfig(**cfg), ctx)
        tr.next_batch()
        tr._dp_g1()
        tr._dp_g2()
        torch.cuda.synchronize()
        assert tr.hstep.fc_path == ("hand_f8" if hand == "1" else "library")
        trs.append(tr)
    a, b = trs
    assert torch.allclose(a.hloss, b.hloss, rtol=1e-2), (a.hloss, b.hloss)
    ga, gb = a.hdce.space.grad, b.hdce.space.grad
    sp = a.hdce.space
    for name, p in zip(sp.names, sp.params):
        sl = sp.slice_of(p)
        x, y = ga[sl], gb[sl]
        assert float((x - y).abs().max()) <= 3e-2 * float(y.abs().max()) + 1e-8, name


@pytest.mark.parametrize("cfg,I,J,K", [(1, 2304, 4096, 2048), (2, 2048, 4096, 2304), (2, 256, 256, 256), (1, 144, 128, 512)])
@pytest.mark.parametrize("f32", [False, True])
def test_gemm_nt_f8_matches_fp32(cuda, cfg, I, J, K, f32):
    """The fp8 backward GEMM form (MX-scaled e4m3 MFMA, two separate device scales) == the fp32 product of
    the same dequantised operands; transpose_u8 is an exact byte transpose."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import gemm_nt_f8, transpose_u8
    torch.manual_seed(3)
    P = torch.randn(I, K, device=cuda)
    Q = torch.randn(J, K, device=cuda) * K ** -0.5
    sp, sq = float(P.abs().max()) / 448.0, float(Q.abs().max()) / 448.0
    P8, Q8 = (P / sp).to(torch.float8_e4m3fn), (Q / sq).to(torch.float8_e4m3fn)
    C = gemm_nt_f8(P8, Q8, torch.tensor([sp], device=cuda), torch.tensor([sq], device=cuda),
                   out_dtype=torch.float32 if f32 else torch.bfloat16, cfg=cfg)
    ref = (P8.float() * sp) @ (Q8.float() * sq).t()
    torch.cuda.synchronize()
    assert _rel(C, ref) < (1e-4 if f32 else 8e-3), _rel(C, ref)
    if I % 64 == 0 and K % 256 == 0:
        T = transpose_u8(P8)
        assert torch.equal(T.view(torch.uint8), P8.view(torch.uint8).t().contiguous())


def test_flagship_fp8_backward_matches_bf16_backward(cuda, monkeypatch):
    """fp8 estimator, full shape (M = 2304): the e4m3 FC weight / data gradients (MX-scaled NT GEMMs over the
    transposed e4m3 copies the loss epilogue and the byte transposes write) vs the bf16 gradient GEMMs, same
    forward, dY scale calibrated from the bf16 run: every HDCE gradient agrees to e4m3 accuracy."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (FlagshipConfig,
                                                                                                FlagshipTrainer)
    ctx = DistContext(device=cuda)
    cfg = dict(batch=256, data_len=600, hip_graphs=False, use_quantumnat=False, stream_mode="serial", dtype="fp8")
    trs = {}
    for bwd in ("0", "1"):
        monkeypatch.setattr(KNOBS, "f8_bwd", bwd == "1")
        trs[bwd] = FlagshipTrainer(FlagshipConfig(**cfg), ctx)
    b16, b8 = trs["0"], trs["1"]
    b16.next_batch()
    b16._dp_g1()
    b16._dp_g2()
    torch.cuda.synchronize()
    assert not getattr(b16.hstep, "_f8_bwd", False)
    dY = b16.hstep._dYW[0]
    # the trainer primed the dY scale itself (FlagshipTrainer._prime_fp8: a bf16-gradient pass on the same
    # first batch), so the DEFAULT state is calibrated -- no set_from_tensor here
    want = float(dY.abs().amax()) * 2.0 / 448.0
    assert abs(float(b8.hdce.fp8_scales.scale[6]) - want) <= 1e-6 * want, (float(b8.hdce.fp8_scales.scale[6]), want)
    b8.next_batch()
    b8._dp_g1()
    b8._dp_g2()
    torch.cuda.synchronize()
    assert b8.hstep._f8_bwd
    assert torch.equal(b8.hloss, b16.hloss)
    assert float(b8.hdce.fp8_scales.scale[6]) != 1.0
    ga, gb = b8.hdce.space.grad, b16.hdce.space.grad
    sp = b8.hdce.space
    for name, p in zip(sp.names, sp.params):
        sl = sp.slice_of(p)
        x, y = ga[sl].float(), gb[sl].float()
        cos = float(torch.nn.functional.cosine_similarity(x.flatten(), y.flatten(), dim=0))
        assert cos > 0.99, (name, cos)
        assert float((x - y).abs().max()) <= 0.15 * float(y.abs().max()) + 1e-8, name


@pytest.mark.parametrize("cfg", [0, 1])
@pytest.mark.parametrize("M,N,K", [(2304, 2048, 4096), (2304, 256, 512), (256, 256, 256)])
def test_gemm_f8_grads_from_row_major(cuda, M, N, K, cfg):
    """The fp8 backward GEMMs on the row-major e4m3 tensors (i-contiguous operands through ds_read_b64_tr_b8):
    dW = s s dY8^T A8 (fp32) and dA = s s dY8 W8 (bf16) == the fp32 products of the same dequantised operands;
    one-hot operands check the layouts exactly.  cfg 1: the same tiles with producer waves."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import gemm_dgrad_f8, gemm_wgrad_f8
    torch.manual_seed(4)
    q = lambda t, s: (t / s).to(torch.float8_e4m3fn)
    dY, A, W = torch.randn(M, N, device=cuda), torch.randn(M, K, device=cuda), torch.randn(N, K, device=cuda)
    sy, sa, sw = (float(t.abs().max()) / 448.0 for t in (dY, A, W))
    dY8, A8, W8 = q(dY, sy), q(A, sa), q(W, sw)
    t = lambda v: torch.tensor([v], device=cuda)
    dW = torch.empty(N, K, device=cuda)
    gemm_wgrad_f8(dY8, A8, t(sy), t(sa), out=dW, cfg=cfg)
    ref_w = (dY8.float() * sy).t() @ (A8.float() * sa)
    torch.cuda.synchronize()
    assert _rel(dW, ref_w) < 1e-4, _rel(dW, ref_w)
    if M % 144 == 0:
        dA = gemm_dgrad_f8(dY8, W8, t(sy), t(sw), cfg=cfg)
        ref_a = (dY8.float() * sy) @ (W8.float() * sw)
        torch.cuda.synchronize()
        assert _rel(dA, ref_a) < 8e-3, _rel(dA, ref_a)
    # exact layout: one-hot dY picks rows of A / W
    oh = torch.zeros(M, N, device=cuda)
    oh[M - 1, 3] = 1.0
    oh[5, N - 2] = 2.0
    gemm_wgrad_f8(oh.to(torch.float8_e4m3fn), A8, t(1.0), t(1.0), out=dW, cfg=cfg)
    torch.cuda.synchronize()
    assert torch.equal(dW[3], A8[M - 1].float()) and torch.equal(dW[N - 2], 2 * A8[5].float())
    assert float(dW[4].abs().sum()) == 0.0

