"""HIP kernel numerics on a real MI355X vs fp32/fp64 CPU references of the same op."""
import math

import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.nmse import StreamNMSE
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.optim import FlatParamSpace, FusedOptimizer
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.quantum import qsim

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8, 9, 10])
@pytest.mark.parametrize("L", [1, 3])
def test_qsim_hip_matches_cpp(cuda, n, L):
    g = torch.Generator().manual_seed(100 * n + L)
    B = 37 if n < 9 else 13  # not a multiple of samples-per-wave
    x = torch.rand(B, n, generator=g) * 2 - 1
    w = torch.rand(L, n, 2, generator=g) * 2 * math.pi
    gE = torch.randn(B, n, generator=g)
    xc, wc = x.clone().requires_grad_(), w.clone().requires_grad_()
    Ec = qsim(xc, wc, "cpu")
    (Ec * gE).sum().backward()
    xg, wg = x.to(cuda).requires_grad_(), w.to(cuda).requires_grad_()
    Eg = qsim(xg, wg, "hip")
    (Eg * gE.to(cuda)).sum().backward()
    torch.cuda.synchronize()
    assert torch.allclose(Eg.cpu(), Ec, atol=2e-5), (Eg.cpu() - Ec).abs().max()
    assert torch.allclose(xg.grad.cpu(), xc.grad, atol=5e-5), (xg.grad.cpu() - xc.grad).abs().max()
    assert torch.allclose(wg.grad.cpu(), wc.grad, atol=5e-4 * max(1, B / 16)), (wg.grad.cpu() - wc.grad).abs().max()


@pytest.mark.parametrize("n,L,B", [(11, 3, 9), (12, 3, 7), (13, 2, 5), (14, 3, 4), (16, 3, 3), (16, 8, 2),
                                   (12, 3, 1000), (11, 2, 800)])
def test_qsim_big_hip_matches_cpp(cuda, n, L, B):
    """Workgroup-per-sample kernels (qsim_big.hip): LDS-resident (n<=12 bwd, n<=13 fwd) and HBM paths."""
    g = torch.Generator().manual_seed(7 * n + L)
    x = torch.rand(B, n, generator=g) * 2 - 1
    w = torch.rand(L, n, 2, generator=g) * 2 * math.pi
    gE = torch.randn(B, n, generator=g)
    xc, wc = x.clone().requires_grad_(), w.clone().requires_grad_()
    Ec = qsim(xc, wc, "cpu")
    (Ec * gE).sum().backward()
    xg, wg = x.to(cuda).requires_grad_(), w.to(cuda).requires_grad_()
    Eg = qsim(xg, wg, "hip")
    (Eg * gE.to(cuda)).sum().backward()
    torch.cuda.synchronize()
    assert torch.allclose(Eg.cpu(), Ec, atol=5e-5), (Eg.cpu() - Ec).abs().max()
    assert torch.allclose(xg.grad.cpu(), xc.grad, atol=2e-4), (xg.grad.cpu() - xc.grad).abs().max()
    assert torch.allclose(wg.grad.cpu(), wc.grad, atol=1e-3), (wg.grad.cpu() - wc.grad).abs().max()


def test_qsim_big_hip_groups(cuda):
    n, L, G, b = 12, 3, 3, 4
    torch.manual_seed(1)
    x = torch.rand(G * b, n) * 2 - 1
    w = torch.rand(G, L, n, 2) * 6.28
    Eg = qsim(x.to(cuda), w.to(cuda), "hip").cpu()
    Ec = torch.cat([qsim(x[i * b:(i + 1) * b], w[i], "cpu") for i in range(G)])
    assert torch.allclose(Eg, Ec, atol=5e-5)


def test_qsim_hip_large_batch_and_groups(cuda):
    n, L, G, b = 8, 3, 9, 256
    torch.manual_seed(0)
    x = (torch.rand(G * b, n) * 2 - 1)
    w = torch.rand(G, L, n, 2) * 6.28
    Eg = qsim(x.to(cuda), w.to(cuda), "hip").cpu()
    Ec = torch.cat([qsim(x[i * b:(i + 1) * b], w[i], "cpu") for i in range(G)])
    assert torch.allclose(Eg, Ec, atol=2e-5)
    # grouped gradient: master weights receive the sum over groups
    m = torch.rand(L, n, 2).to(cuda).requires_grad_()
    noise = torch.randn(G, L, n, 2, device=cuda) * 0.01
    xs = x.to(cuda).requires_grad_()
    qsim(xs, m.unsqueeze(0) + noise, "hip").sum().backward()
    mc = m.detach().cpu().requires_grad_()
    xc = x.clone().requires_grad_()
    qsim(xc, mc.unsqueeze(0) + noise.cpu(), "cpu").sum().backward()
    assert torch.allclose(m.grad.cpu(), mc.grad, rtol=1e-3, atol=1e-2)
    assert torch.allclose(xs.grad.cpu(), xc.grad, atol=5e-5)


def test_qsim_hip_graph_capture(cuda):
    n, L, B = 8, 3, 512
    x = (torch.rand(B, n, device=cuda) * 2 - 1).requires_grad_()
    w = torch.rand(L, n, 2, device=cuda).requires_grad_()
    out = torch.zeros(1, device=cuda)

    def body():
        x.grad = None
        w.grad = None
        E = qsim(x, w, "hip")
        E.sum().backward()
        out.copy_(E.sum())

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    ref = out.clone()
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph):
        body()
    gph.replay()
    torch.cuda.synchronize()
    assert torch.allclose(out, ref)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_stream_nmse_hip_vs_cpu(cuda, dt):
    torch.manual_seed(1)
    S, b, C = 9, 40, 2048
    rs = torch.arange(S).repeat_interleave(b)[torch.randperm(S * b)]
    Y = torch.randn(S * b, C).to(dt).float()
    Lb = torch.randn(S * b, C)
    Pf = torch.randn(S * b, C)
    cpu = StreamNMSE(rs, S)
    lc, gc = cpu(Y, Lb, Pf)
    gpu = StreamNMSE(rs.to(cuda), S)
    lg, gg = gpu(Y.to(cuda).to(dt), Lb.to(cuda), Pf.to(cuda), out_dtype=torch.float32)
    assert torch.allclose(lg.cpu(), lc, rtol=1e-5)
    assert torch.allclose(gg.cpu(), gc, rtol=1e-4, atol=1e-9)
    # reference definition: mean over streams of per-stream global ratios
    ref = sum(((Y[rs == s] - Lb[rs == s]) ** 2).sum() / (Lb[rs == s] ** 2).sum() for s in range(S)) / S
    assert torch.allclose(lg[0].cpu(), ref, rtol=1e-5)
    assert float(gpu.skip.item()) == 0.0
    # fused reduce+finalize launch == the two-launch path
    gpu2 = StreamNMSE(rs.to(cuda), S)
    l2 = gpu2.sums_finalize(Y.to(cuda).to(dt), Lb.to(cuda), Pf.to(cuda))
    assert torch.allclose(l2, lg, rtol=1e-6) and torch.allclose(gpu2.coef, gpu.coef, rtol=1e-6)
    # NaN guard raises the flag
    Yn = Y.clone()
    Yn[3, 7] = float("nan")
    gpu2.sums_finalize(Yn.to(cuda).to(dt), Lb.to(cuda), Pf.to(cuda))
    assert float(gpu2.skip.item()) == 1.0
    # gradient + fused FC bias gradient (column sums of dY) == the separate passes
    gpu3 = StreamNMSE(rs.to(cuda), S)
    gpu3.sums_finalize(Y.to(cuda).to(dt), Lb.to(cuda), Pf.to(cuda))
    bg = torch.full((C,), 7.0, device=cuda)   # overwritten
    dY3 = gpu3.grad_bias(Y.to(cuda).to(dt), Lb.to(cuda), bg, out_dtype=torch.bfloat16)
    dY1 = gpu3.grad(Y.to(cuda).to(dt), Lb.to(cuda), out_dtype=torch.bfloat16)
    assert torch.equal(dY3, dY1)
    ref_b = (gpu3.coef[gpu3._rs_long][:, None] * (Y.to(cuda).to(dt).float() - Lb.to(cuda))).sum(0)
    assert torch.allclose(bg, ref_b, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("kind", ["adam", "adamw", "sgd"])
def test_fused_optimizer_hip_vs_torch(cuda, kind):
    torch.manual_seed(2)
    shapes = [(33, 7), (5,), (64, 3, 3, 3)]
    ref_params = [torch.nn.Parameter(torch.randn(s, device=cuda)) for s in shapes]
    our_params = [torch.nn.Parameter(p.detach().clone()) for p in ref_params]
    space = FlatParamSpace([(f"p{i}", p) for i, p in enumerate(our_params)], cuda)
    if kind == "adam":
        ref = torch.optim.Adam(ref_params, lr=1e-2)
        opt = FusedOptimizer(space, "adam", lr=1e-2)
    elif kind == "adamw":
        ref = torch.optim.AdamW(ref_params, lr=1e-2, weight_decay=0.01)
        opt = FusedOptimizer(space, "adamw", lr=1e-2, weight_decay=0.01)
    else:
        ref = torch.optim.SGD(ref_params, lr=1e-2, momentum=0.9)
        opt = FusedOptimizer(space, "sgd", lr=1e-2, momentum=0.9)
    for it in range(5):
        grads = [torch.randn(s, device=cuda) for s in shapes]
        for p, g in zip(ref_params, grads):
            p.grad = g.clone()
        for p, g in zip(our_params, grads):
            p.grad.copy_(g)
        ref.step()
        opt.step()
    for a, b in zip(ref_params, our_params):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (a - b).abs().max()


def test_fused_optimizer_skip_and_prune(cuda):
    p = torch.nn.Parameter(torch.ones(100, device=cuda))
    space = FlatParamSpace([("p", p)], cuda)
    opt = FusedOptimizer(space, "adamw", lr=0.1, weight_decay=0.01, prune_thr=0.5)
    p.grad.copy_(torch.linspace(-1, 1, 100, device=cuda))
    skip = torch.ones(1, dtype=torch.float32, device=cuda)
    opt.step(skip=skip)
    assert torch.equal(p.detach(), torch.ones(100, device=cuda)) and opt.step_t.item() == 0
    skip.zero_()
    opt.step(skip=skip)
    small = torch.linspace(-1, 1, 100).abs() <= 0.5
    assert opt.pruned_count(1) == int(small.sum())
    moved = (p.detach().cpu() - (1 - 0.1 * 0.01)).abs() > 1e-6
    assert torch.equal(moved, ~small)


def test_step_gather_hip_matches_host(cuda):
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.datasets import make_dml_stores
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.gather import StepGather
    tr, _ = make_dml_stores(60, 128, 10, 0.9, "cpu", synthetic=True, base_seed=5)
    tr = tr.shard(1, 2)
    idx = torch.randperm(tr.n)[:7]
    host = StepGather(3, 3, 7, 16, 8, "cpu")
    host(tr, idx)
    dev = StepGather(3, 3, 7, 16, 8, cuda)
    dev(tr.to(cuda), idx.to(cuda))
    torch.cuda.synchronize()
    assert torch.equal(dev.x1.cpu(), host.x1) and torch.equal(dev.xq.cpu(), host.xq)
    # (the device store is contiguous, the host shard is a view: compare addressed rows)
    d = tr.to(cuda)
    sr = d.Hlabel.stride(0) // 2048
    o = dev.rowoff.long().cpu()
    sr_h = tr.Hlabel.stride(0) // 2048
    oh = host.rowoff.long()
    assert torch.equal(d.Hlabel.cpu()[o // sr, o % sr], tr.Hlabel[oh // sr_h, oh % sr_h])


def test_gather_device_cursor(cuda):
    """qd_gather_cursor: batch = perm[*cur : *cur + B] and *cur advances by B in-kernel (last-workgroup
    protocol), for the HDCE half (x1 + rowoff) and the classifier half (xq) with separate cursors."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.datasets import make_dml_stores
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.gather import StepGather
    st, _ = make_dml_stores(60, 128, 10, 0.9, "cpu", synthetic=True, base_seed=5)
    d = st.to(cuda)
    B = 7
    perm = torch.randperm(d.n, device=cuda)
    cur = torch.zeros(2, dtype=torch.int32, device=cuda)
    done = torch.zeros(2, dtype=torch.int32, device=cuda)
    g = StepGather(3, 3, B, 16, 8, cuda)
    ref = StepGather(3, 3, B, 16, 8, cuda)
    cols = d.Hlabel.shape[-1]
    rp = (d.Hlabel.pow(2).sum(-1).reshape(-1).contiguous(), d.Hperf.pow(2).sum(-1).reshape(-1).contiguous())
    g.rowpow = rp   # (contiguous store: rowoff row space = s * N + n)
    assert d.Hlabel.stride(0) == d.n * cols
    for k in range(5):
        g.from_cursor(d, perm, cur[0:1], done[0:1], hdce=True, classifier=False)
        g.from_cursor(d, perm, cur[1:2], done[1:2], hdce=False, classifier=True)
        ref(d, perm[k * B:(k + 1) * B].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(g.x1, ref.x1) and torch.equal(g.xq, ref.xq) and torch.equal(g.rowoff, ref.rowoff), k
        o = g.rowoff.long()
        assert torch.equal(g.rowden[:, 0], rp[0][o]) and torch.equal(g.rowden[:, 1], rp[1][o])
        assert cur.tolist() == [(k + 1) * B] * 2 and done.tolist() == [0, 0]
    # an exhausted cursor never reads past the permutation: it restarts at 0
    cur.fill_(d.n - 3)
    g.from_cursor(d, perm, cur[0:1], done[0:1], hdce=True, classifier=True)
    ref(d, perm[:B].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(g.x1, ref.x1) and int(cur[0]) == B


def test_fused_optimizer_tick_and_shadow(cuda):
    """Step counter ticks exactly once per launch (last-workgroup pattern) across many workgroups,
    never on a skipped step, and the bf16 shadow tracks the updated weights."""
    torch.manual_seed(3)
    p = torch.nn.Parameter(torch.randn(3_000_001, device=cuda))
    sp = FlatParamSpace([("p", p)], cuda)
    opt = FusedOptimizer(sp, "adam", lr=1e-3)
    sh = opt.attach_shadow(0, 2_000_000)
    skip = torch.zeros(1, device=cuda)
    for i in range(5):
        sp.grad.normal_()
        opt.step(skip=skip)
    skip.fill_(1.0)
    opt.step(skip=skip)
    torch.cuda.synchronize()
    assert float(opt.step_t.item()) == 5.0 and int(opt.done.item()) == 0
    assert torch.equal(sh, sp.flat[:2_000_000].to(torch.bfloat16))


@pytest.mark.parametrize("accumulate", [False, True])
def test_slab_batch_multi_reduction(cuda, accumulate):
    """One launch reducing several slabs (vector and scalar-width jobs) == torch sums."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.slabsum import SlabBatch
    torch.manual_seed(3)
    shapes = [(3, 48, 576), (1, 256, 48), (1, 37, 30), (2, 5, 9218)]   # (groups, rows, width)
    slabs = [torch.randn(g, r, w, device=cuda) for g, r, w in shapes]
    outs = [torch.randn(g, w, device=cuda) for g, _, w in shapes]
    refs = [s.sum(1) + (o if accumulate else 0) for s, o in zip(slabs, outs)]
    b = SlabBatch()
    for s, o, (g, r, w) in zip(slabs, outs, shapes):
        b.add(s, o, g, r, w)
    b.launch(accumulate, nat.stream_ptr(cuda))
    torch.cuda.synchronize()
    for o, ref in zip(outs, refs):
        assert torch.allclose(o, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("with_perf", [True, False])
def test_nmse_fused_matches_two_pass(cuda, with_perf):
    """qd_nmse_fused (one pass over Y/labels + finish) == the row-sum / finalize / grad_bias kernels and
    an fp32 torch reference: loss, loss_perf, dY, bias gradient; labels read through rowoff from a
    strided store view."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.nmse import StreamNMSE
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel
    torch.manual_seed(3)
    E, U, B, cols, N = 3, 3, 32, 2048, 50
    S = E * U
    full_l = torch.randn(S, 2 * N, cols, device=cuda)
    full_p = full_l + 0.3 * torch.randn_like(full_l)
    L, P = full_l[:, 10:10 + N], full_p[:, 10:10 + N]          # strided (shard-like) views
    sr = L.stride(0) // cols
    idx = torch.randint(0, N, (B,), device=cuda)
    u = torch.arange(U, device=cuda).view(U, 1, 1)
    e = torch.arange(E, device=cuda).view(1, 1, E)
    s = (e * U + u).expand(U, B, E)
    rowoff = (s * sr + idx.view(1, B, 1)).reshape(-1).to(torch.int32)
    rs = HDCEModel.row_stream(E, U, B, cuda)
    rows = U * B * E
    Y = (torch.randn(rows, cols, device=cuda) * 0.8).bfloat16()
    a, b = StreamNMSE(rs, S, cols), StreamNMSE(rs, S, cols)
    a.rowoff = b.rowoff = rowoff
    perf = P if with_perf else None
    la = a.sums_finalize(Y, L, perf).clone()
    bg_a = torch.empty(cols, device=cuda)
    dYa = a.grad_bias(Y, L, bg_a, out_dtype=torch.bfloat16)
    bg_b = torch.full((cols,), 1e30, device=cuda)
    dYb = b.fused(Y, L, perf, bg_b, (E, U, B), out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.allclose(b.loss, la, rtol=1e-5, atol=1e-7), (b.loss, la)
    assert float(b.skip) == 0.0
    assert (dYa.float() - dYb.float()).abs().max() <= 1e-2 * dYa.float().abs().max()
    assert torch.allclose(bg_a, bg_b, rtol=1e-4, atol=1e-6)
    # fp32 reference
    lab = L[(rowoff // sr).long(), (rowoff % sr).long()]
    Yf = Y.float()
    ref = 0.0
    for k in range(S):
        m = rs == k
        ref += float(((Yf[m] - lab[m]) ** 2).sum() / (lab[m] ** 2).sum())
    assert abs(float(b.loss[0]) - ref / S) <= 1e-5 * abs(ref / S)
    # NaN guard
    Y[5, 7] = float("nan")
    b.fused(Y, L, perf, bg_b, (E, U, B), out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert float(b.skip) == 1.0


@pytest.mark.parametrize("n,L,B", [(12, 3, 7), (14, 3, 5), (16, 2, 3), (13, 1, 4), (12, 3, 1100)])
def test_qsim_big_saved_state_backward(cuda, n, L, B):
    """qsim_big with the forward's psi_final kept for the adjoint backward (no recompute) == the
    recomputing backward: same E, dx and weight-gradient slab (to fp32 rounding: the fused forward
    generates the layer-0 product state in a different code site than the backward's recompute)."""
    import ctypes
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    lib = nat.hip_lib()
    _p, _i = ctypes.c_void_p, ctypes.c_int
    torch.manual_seed(n)
    x = torch.rand(B, n, device=cuda) * 3.0
    w = torch.rand(L, n, 2, device=cuda) * 6.28
    gE = torch.randn(B, n, device=cuda)
    grid = nat.fn(lib, "qd_qsim_big_grid", [_i])(B)
    wsb = nat.fn(lib, "qd_qsim_big_workspace", [_i, _i, _i], ctypes.c_longlong)(n, grid, 1)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=cuda)
    ps = torch.empty(B * (8 << n), dtype=torch.uint8, device=cuda)
    f = nat.fn(lib, "qd_qsim_big_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
    b = nat.fn(lib, "qd_qsim_big_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
    st = nat.stream_ptr(cuda)
    out = []
    for save in (False, True):
        E = torch.empty(B, n, device=cuda)
        dx = torch.empty(B, n, device=cuda)
        slab = torch.empty(grid, 2 * n * L, device=cuda)
        sp = nat.ptr(ps) if save else None
        nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(E), B, n, L, 0, nat.ptr(ws), sp, st), "fwd")
        nat.check(b(nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, n, L, 0, nat.ptr(ws), sp, st),
                  "bwd")
        torch.cuda.synchronize()
        out.append((E, dx, slab))
    for a, c in zip(*out):
        assert torch.allclose(a, c, rtol=1e-5, atol=1e-6), float((a - c).abs().max())


@pytest.mark.parametrize("n,L,B", [(4, 3, 37), (6, 2, 9), (8, 3, 33), (10, 3, 5)])
def test_qsim_saved_state_backward(cuda, n, L, B):
    """Register-resident simulator: the backward from the forward's saved final state == the
    recomputing backward (to fp32 rounding: the two kernels' circuit code may contract differently)."""
    import ctypes
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    lib = nat.hip_lib()
    _p, _i = ctypes.c_void_p, ctypes.c_int
    torch.manual_seed(n)
    x = torch.rand(B, n, device=cuda) * 3.0
    w = torch.rand(L, n, 2, device=cuda) * 6.28
    gE = torch.randn(B, n, device=cuda)
    rows = nat.fn(lib, "qd_qsim_bwd_grid", [_i, _i])(n, B)
    ps = torch.empty(B * (8 << n), dtype=torch.uint8, device=cuda)
    st = nat.stream_ptr(cuda)
    out = []
    for save in (False, True):
        E = torch.empty(B, n, device=cuda)
        dx = torch.empty(B, n, device=cuda)
        slab = torch.empty(rows, 2 * n * L, device=cuda)
        if save:
            f = nat.fn(lib, "qd_qsim_fwd_save", [_p, _p, _p, _i, _i, _i, _i, _p, _p])
            b = nat.fn(lib, "qd_qsim_bwd_saved", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p])
            nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(E), B, n, L, 0, nat.ptr(ps), st), "fwd")
            nat.check(b(nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, n, L, 0, nat.ptr(ps), st),
                      "bwd")
        else:
            f = nat.fn(lib, "qd_qsim_fwd", [_p, _p, _p, _i, _i, _i, _i, _p])
            b = nat.fn(lib, "qd_qsim_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p])
            nat.check(f(nat.ptr(x), nat.ptr(w), nat.ptr(E), B, n, L, 0, st), "fwd")
            nat.check(b(nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx), nat.ptr(slab), B, n, L, 0, st), "bwd")
        torch.cuda.synchronize()
        out.append((E, dx, slab))
    for a, c in zip(*out):
        assert torch.allclose(a, c, rtol=1e-5, atol=1e-6), float((a - c).abs().max())


@pytest.mark.parametrize("n,L,B,G", [(13, 2, 6, 2), (14, 3, 4, 1), (15, 3, 6, 3), (16, 3, 4, 2), (16, 5, 2, 1)])
def test_qsim_stream_matches_per_sample_kernel(cuda, n, L, B, G):
    """Streamed simulator (qsim_stream.hip: one workgroup per (sample, brick) per pass, ring as an LDS
    scatter; the backward reads the forward's kept pass-A states and generates layer 0) == the
    workgroup-per-sample kernels (qsim_big.hip): E, dx and the summed weight gradient, per-group
    (QuantumNAT) weights, with and without the forward's kept states."""
    import ctypes
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    lib = nat.hip_lib()
    _p, _i = ctypes.c_void_p, ctypes.c_int
    torch.manual_seed(n + 10 * L)
    x = torch.rand(B * G, n, device=cuda) * 3.0 - 1.5
    w = torch.rand(G, L, n, 2, device=cuda) * 6.28
    gE = torch.randn(B * G, n, device=cuda)
    st = nat.stream_ptr(cuda)
    BB = B * G
    # per-sample kernels
    grid = nat.fn(lib, "qd_qsim_big_grid", [_i])(BB)
    wsb = nat.fn(lib, "qd_qsim_big_workspace", [_i, _i, _i], ctypes.c_longlong)(n, grid, 1)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=cuda)
    E0, dx0 = torch.empty(BB, n, device=cuda), torch.empty(BB, n, device=cuda)
    slab0 = torch.empty(grid, 2 * n * L, device=cuda)
    nat.check(nat.fn(lib, "qd_qsim_big_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])(
        nat.ptr(x), nat.ptr(w), nat.ptr(E0), BB, n, L, B, nat.ptr(ws), None, st), "big fwd")
    nat.check(nat.fn(lib, "qd_qsim_big_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])(
        nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx0), nat.ptr(slab0), BB, n, L, B, nat.ptr(ws), None, st), "big bwd")
    assert bool(nat.fn(lib, "qd_qsim_stream_ok", [_i, _i])(n, L))
    rows = nat.fn(lib, "qd_qsim_stream_rows", [_i])(BB)
    wss = nat.fn(lib, "qd_qsim_stream_workspace", [_i, _i, _i, _i], ctypes.c_longlong)(n, BB, L, 1)
    ws2 = torch.empty(wss, dtype=torch.uint8, device=cuda)
    ps = torch.empty(nat.fn(lib, "qd_qsim_stream_save_bytes", [_i, _i, _i], ctypes.c_longlong)(n, BB, L),
                     dtype=torch.uint8, device=cuda)
    sf = nat.fn(lib, "qd_qsim_stream_fwd", [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
    sb = nat.fn(lib, "qd_qsim_stream_bwd", [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p])
    for save in (True, False):
        E1, dx1 = torch.empty(BB, n, device=cuda), torch.empty(BB, n, device=cuda)
        slab1 = torch.full((rows, 2 * n * L), float("nan"), device=cuda)
        nat.check(sf(nat.ptr(x), nat.ptr(w), nat.ptr(E1), BB, n, L, B, nat.ptr(ws2), nat.ptr(ps) if save else None, st),
                  "stream fwd")
        nat.check(sb(nat.ptr(x), nat.ptr(w), nat.ptr(gE), nat.ptr(dx1), nat.ptr(slab1), BB, n, L, B, nat.ptr(ws2),
                     nat.ptr(ps) if save else None, st), "stream bwd")
        torch.cuda.synchronize()
        assert not bool(torch.isnan(slab1).any()), "every slab element written"
        assert torch.allclose(E1, E0, atol=2e-5), float((E1 - E0).abs().max())
        assert torch.allclose(dx1, dx0, atol=1e-4), float((dx1 - dx0).abs().max())
        g0, g1 = slab0.sum(0), slab1.sum(0)
        assert torch.allclose(g1, g0, atol=2e-4 * B * G, rtol=1e-4), float((g1 - g0).abs().max())


def _mfma_fwd(cuda, x, w, wgroup, save):
    import ctypes
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    lib = nat.hip_lib()
    _p, _i = ctypes.c_void_p, ctypes.c_int
    G, L = w.shape[0], w.shape[1]
    B = x.shape[0]
    nh = nat.fn(lib, "qd_qsim_mfma_ops_halves", [_i, _i], ctypes.c_longlong)(G, L)
    ops = torch.empty(nh, dtype=torch.float16, device=cuda)
    E = torch.empty(B, 8, device=cuda)
    ps = torch.zeros(B * 256 * 2, device=cuda) if save else None
    st = nat.stream_ptr(cuda)
    nat.check(nat.fn(lib, "qd_qsim_mfma_prep", [_p, _p, _i, _i, _p])(nat.ptr(w), nat.ptr(ops), G, L, st), "prep")
    nat.check(nat.fn(lib, "qd_qsim_mfma_fwd", [_p, _p, _p, _p, _i, _i, _i, _p, _p])(
        nat.ptr(x), nat.ptr(w), nat.ptr(ops), nat.ptr(E), B, L, wgroup, nat.ptr(ps) if save else None, st), "fwd")
    return E, ps


@pytest.mark.parametrize("L,G,b", [(2, 1, 37), (3, 9, 16), (5, 3, 7)])
def test_qsim_mfma_forward_matches_register_kernel(cuda, L, G, b):
    """8-qubit forward on the matrix cores (qsim_mfma.hip: Kronecker-factored layer unitaries as
    complex MFMA GEMMs, fp16 hi/lo split) == the register kernel (qsim.hip) and the fp64 CPU oracle:
    <Z> and the saved final state (the adjoint backward's input)."""
    import ctypes
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    lib = nat.hip_lib()
    _p, _i = ctypes.c_void_p, ctypes.c_int
    torch.manual_seed(L * 10 + G)
    B = G * b
    x = torch.rand(B, 8, device=cuda) * 2 - 1
    w = torch.rand(G, L, 8, 2, device=cuda) * 6.28
    E1, ps1 = _mfma_fwd(cuda, x, w, b if G > 1 else 0, True)
    E0 = torch.empty(B, 8, device=cuda)
    ps0 = torch.zeros(B * 256 * 2, device=cuda)
    nat.check(nat.fn(lib, "qd_qsim_fwd_save", [_p, _p, _p, _i, _i, _i, _i, _p, _p])(
        nat.ptr(x), nat.ptr(w), nat.ptr(E0), B, 8, L, b if G > 1 else 0, nat.ptr(ps0), nat.stream_ptr(cuda)), "reg")
    torch.cuda.synchronize()
    assert torch.allclose(E1, E0, atol=3e-6), float((E1 - E0).abs().max())
    assert torch.allclose(ps1, ps0, atol=2e-6), float((ps1 - ps0).abs().max())
    Ec = torch.cat([qsim(x[i * b:(i + 1) * b].cpu(), w[i].cpu(), "cpu") for i in range(G)])
    assert torch.allclose(E1.cpu(), Ec, atol=5e-6), float((E1.cpu() - Ec).abs().max())
