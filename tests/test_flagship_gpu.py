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
    tr._dp_g1()
    tr._dp_g2()
    ref = [g.clone() for g in _views(tr)]
    # poison every parameter gradient, then the write-mode step must reproduce ref exactly
    for g in _views(tr):
        g.fill_(1e30)
    tr.hstep.writes_grads, tr.cstep.writes_grads = True, True
    tr.cur.zero_()   # same batch again (the gather advanced the device cursor)
    tr._dp_g1()
    tr._dp_g2()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(_views(tr), ref)):
        assert torch.isfinite(a).all() and a.abs().max() < 1e29, i
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-7), (i, float((a - b).abs().max()))


def _opts(opt: str) -> dict:
    """'conv' / 'fcnext' (the part of a test mode after '+') -> the FlagshipConfig options they stand for"""
    return {"conv": {"qsc_start": "conv"}, "fcnext": {"fc_adam_next": 256}, "": {}}[opt]


def _all_state(tr):
    return [tr.hdce.space.flat, tr.qspace.flat, tr.hopt.m, tr.hopt.v, tr.qopt.m, tr.qopt.v,
            tr.hdce.fc_shadow] + list(tr.hdce.run_mean) + list(tr.hdce.run_var)


@pytest.mark.parametrize("mode,split,k", [("dagq", True, 1), ("dagq", False, 1), ("dagq", False, 3), ("indep", False, 3),
                                         ("indep+conv", False, 3), ("indep+fcnext", False, 3)])
def test_multistream_graph_matches_serial_eager(cuda, mode, split, k):
    """The multi-stream step (captured in one graph, or the 5-graph DP plan) computes exactly what the
    single-stream eager step computes: every kernel is deterministic (slab reductions, no float
    atomics) and the DAG only reorders independent work.  ("indep+conv": the QSC chain of each step starts after
    the HDCE conv forward, FlagshipConfig.qsc_start; "indep+fcnext": the FC weight's Adam overlaps the next step's
    conv forward, FlagshipConfig.fc_adam_next.)"""
    _graph_vs_serial(cuda, mode, split, k)


@pytest.mark.parametrize("mode", ["indep+conv", "indep+fcnext"])
def test_split_plans_match_serial_with_library_fc_forward(cuda, monkeypatch, mode):
    """The split-forward plans with hipBLASLt's FC forward (no hand forward GEMM): the pairing that exposed the QSC
    preprocess forward's lane-dependent conv1 weights under concurrency -- 20-30 of 288 samples, channel 5 of the
    last pool row (lanes 48-63), differed from an eager recompute in every run until the weights were read through
    readfirstlane (csrc/hip/qsc_mfma.hip conv1_half; profiles/r5_55_entries.txt, r5_56_uniform_probe.txt)."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS
    monkeypatch.setattr(KNOBS, "hand_gemm", "wgrad,dgrad")
    dag = _graph_vs_serial(cuda, mode, False, 3)
    assert dag.hstep.fc_path == "library"


def _graph_vs_serial(cuda, mode, split, k):
    ctx = DistContext(device=cuda)
    mode, _, start = mode.partition("+")
    # (the same QSC backward grid on both sides: it fixes the slab reduction order)
    base = dict(batch=32, data_len=800, use_quantumnat=True, qsc_grid_bwd=128)
    ref = FlagshipTrainer(FlagshipConfig(hip_graphs=False, stream_mode="serial", **base), ctx)
    dag = FlagshipTrainer(FlagshipConfig(hip_graphs=True, stream_mode=mode, split_graphs=split,
                                         steps_per_graph=k, **_opts(start), **base), ctx)
    assert dag.streams is not None and ref.streams is None
    assert dag.fc_adam_next == (start == "fcnext")
    dag.capture(preserve=True, k=k)   # (capturing runs warm-up steps; the state is restored)
    dag.capture(preserve=True, k=1)
    for _ in range(4):
        ref.step()
    dag.run(4)                        # k-step replays + single steps for the remainder
    torch.cuda.synchronize()
    assert torch.equal(ref.skip_flags(), dag.skip_flags()) and float(dag.skip_flags().sum()) == 0.0
    for i, (a, b) in enumerate(zip(_all_state(ref), _all_state(dag))):
        if b.numel() != a.numel():   # (the DP plan's HDCE space has a scratch slot at the end: the NaN flag)
            b = b[:a.numel()]
        assert torch.allclose(a.float(), b.float(), rtol=1e-6, atol=1e-7), (i, float((a.float() - b.float()).abs().max()))
    assert torch.allclose(ref.hloss, dag.hloss, rtol=1e-6) and torch.allclose(ref.qloss, dag.qloss, rtol=1e-6)
    assert float(ref.hopt.step_t[0]) == 4.0 and bool((dag.hopt.step_t == 4.0).all())
    return dag


@pytest.mark.parametrize("mode,split,k", [("dagq", False, 4), ("dagq", True, 1), ("indep", False, 4),
                                         ("indep+conv", False, 4), ("indep+fcnext", False, 4)])
def test_shipped_plans_bit_exact_over_12_steps(cuda, mode, split, k):
    """The plans bench.py / the DP path run -- dagq (QSC branch forked and joined every step, k steps per
    replay), indep (the two chains independent for the whole replay, each gathering its own half of the batch)
    and the 5-graph data-parallel plan -- reproduce the same plan run eagerly on one stream BIT FOR BIT over 12
    steps, in every one of 3 fresh trainer pairs (docs/CONCURRENCY.md: round 3's independent-chains plan dagi,
    whose QSC branch read the classifier input the NEXT step's gather rewrote, did not, in 10-25 of 25 trials).
    (The DP plan reduces the FC bias gradient in its own launch, so its reference is the DP plan run eagerly.)"""
    import os
    ctx = DistContext(device=cuda)
    mode, _, start = mode.partition("+")
    base = dict(batch=32, data_len=800, use_quantumnat=True, qsc_grid_bwd=128)
    for trial in range(int(os.environ.get("QDML_BITEXACT_TRIALS", "3"))):   # (more trials: a longer GPU call)
        ref = FlagshipTrainer(FlagshipConfig(hip_graphs=False, stream_mode="serial", split_graphs=split, **base), ctx)
        dag = FlagshipTrainer(FlagshipConfig(hip_graphs=True, stream_mode=mode, split_graphs=split,
                                             steps_per_graph=k, **_opts(start), **base), ctx)
        dag.capture(preserve=True, k=k)
        for rep in range(12 // k):
            for _ in range(k):
                ref.step()
            dag.run(k)
            torch.cuda.synchronize()
            for i, (a, b) in enumerate(zip(_all_state(ref), _all_state(dag))):
                b = b[:a.numel()] if b.numel() != a.numel() else b
                assert torch.equal(a, b), (trial, rep, i, float((a.float() - b.float()).abs().max()))
        assert torch.equal(ref.qloss, dag.qloss) and torch.equal(ref.hloss, dag.hloss)


@pytest.mark.parametrize("plan", ["zero", "allreduce"])
def test_dp_plan_two_ranks_on_one_gpu(tmp_path, plan):
    """The DP execution plan on the GPU (4 graphs, side streams, async bucketed all-reduces) with 2 ranks
    sharing the card over gloo: ranks stay bit-identical step after step and a NaN on one rank makes both
    skip.  (The 8-GPU RCCL run is the driver's; this covers the same code path on one device.)"""
    import os
    import sys
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch import launch
    here = os.path.dirname(os.path.abspath(__file__))
    out = str(tmp_path / "fl")
    rc = launch([sys.executable, os.path.join(here, "dist_scripts", "flagship_dp.py"), out, "cuda"], nproc=2,
                extra_env={"OMP_NUM_THREADS": "2", "QDML_DIST_BACKEND": "gloo", "QDML_DP_PLAN": plan})
    assert rc == 0
    for r in range(2):
        same, skipped, flag = open(f"{out}.{r}").read().split()
        assert same == "1" and skipped == "1" and float(flag) >= 1.0, (r, same, skipped, flag)


def _two_ranks_one_gpu(tmp_path, script, env):
    import os
    import sys
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch import launch
    here = os.path.dirname(os.path.abspath(__file__))
    out = str(tmp_path / "z")
    rc = launch([sys.executable, os.path.join(here, "dist_scripts", script), out, "cuda"], nproc=2,
                extra_env={"OMP_NUM_THREADS": "2", "QDML_DIST_BACKEND": "gloo", **env})
    assert rc == 0
    return [open(f"{out}.{r}").read().split() for r in range(2)]


def test_zero_plan_matches_allreduce_plan_on_gpu(tmp_path):
    """ZeRO-1 FC optimizer == all-reduce plan bit for bit on the GPU DP plan (2 ranks sharing the card over
    gloo): reduce-scatter, Adam on each rank's FC shard writing its slice of the bf16 shadow, all-gather.
    The QSC branch runs on the main stream here (stream_mode serial): with it forked (dagq) the DP plan on a
    SHARED card is not run-to-run deterministic in the QSC weights -- the same plan twice differs as often
    as the two plans do (profiles/r3_03_zero_diag.txt, docs/CONCURRENCY.md); that is the next test."""
    for r, rec in enumerate(_two_ranks_one_gpu(tmp_path, "zero_vs_allreduce.py", {"QDML_STREAM_MODE": "serial"})):
        assert rec[0] == "1", (r, rec)


def test_dp_plan_run_to_run_on_shared_gpu(tmp_path):
    """Two processes sharing one GPU run the same DP plan twice: bit-identical (strict since round 6).  Round 3's
    ~1-in-4 QSC-only mismatch here was the QSC preprocess forward's lanes-48..63 misread, whose cause round 6
    named -- a packed-FP32 FMA reading registers a younger LDS read rewrites, under a co-resident wave's MFMAs
    (csrc/hip/hazard_probe.hip, profiles/r6_03_pkfma_war.txt) -- and removed from the whole library (no packed-FP32
    instructions: _native.NO_PACKED_F32, tests/test_no_packed_f32.py; docs/CONCURRENCY.md)."""
    for r, rec in enumerate(_two_ranks_one_gpu(tmp_path, "zero_vs_allreduce.py", {"QDML_ZV_PLANS": "allreduce,allreduce"})):
        assert rec[0] == "1", (r, rec)


@pytest.mark.parametrize("plan,k,qsc", [("zero", 1, "g2"), ("allreduce", 1, "g2"), ("allreduce", 3, "g2"),
                                        ("zero", 1, "fwd"), ("allreduce", 3, "fwd"), ("allreduce", 1, "indep"),
                                        ("allreduce", 3, "indep")])
def test_dp_one_graph_matches_five_graphs_over_rccl(tmp_path, plan, k, qsc):
    """The DP step captured as ONE graph with its RCCL collectives inside == the 5-graph DP plan (which
    launches the collectives between replays), bit for bit over 6 steps: a real RCCL process group of
    one rank (QDML_FORCE_DIST=1), so the reduce-scatter / all-reduce / all-gather are captured.  k = 3:
    three steps per replay, each step's FC update overlapping the next step's conv forward.  qsc "fwd": the
    one-graph plan's QSC branch forked after the gather (cfg.dp_qsc) -- the same kernels on the same inputs,
    so still bit-exact; qsc "indep" (round 6): the QSC chain independent, its bucket all-reduced at the next step's
    start (DPPlan._dp_run_indep).  (k = 1: the one-graph trainer's phase_times -- clock stamps captured inside the graph
    -- must also fit in its step.)"""
    import os
    import sys
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch import launch
    here = os.path.dirname(os.path.abspath(__file__))
    out = str(tmp_path / "og")
    rc = launch([sys.executable, os.path.join(here, "dist_scripts", "dp_one_graph.py"), out, plan, str(k), qsc], nproc=1,
                extra_env={"OMP_NUM_THREADS": "2", "QDML_FORCE_DIST": "1"})
    assert rc == 0
    rec = open(f"{out}.0").read().split()
    assert rec[0] == "1", rec


def test_bench_two_ranks_one_gpu_reports_phases(tmp_path):
    """`bench.py --gpus 2` self-launches 2 ranks (gloo on one card) and reports dp2 with per-phase times."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update({"QDML_DIST_BACKEND": "gloo", "OMP_NUM_THREADS": "2"})
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "2",
                        "--phase-steps", "3"], capture_output=True, text=True, env=env, timeout=300, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    recs = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(recs) == 1
    r = recs[0]
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2"
    sel = r["config"]["plan_select_ms"]   # (both plans timed at world 2, the faster one benchmarked)
    assert set(sel) == {"zero", "allreduce"} and r["config"]["dp_plan"] == min(sel, key=sel.get)
    assert r["config"]["dp_graph"] == "five"   # (gloo: no captured collectives, so its phases are reported)
    ph = r["phases_ms"]
    assert set(ph) >= {"g1", "g2", "fc_exposed", "fc_adam", "all_gather", "conv_qsc_adam", "step"}
    assert ph["step"] > 0 and ph["g1"] > 0


def test_deferred_loss_finish_matches_finish_launch(cuda):
    """The HDCE loss finish hosted by the conv backward's BN-reduction launch (default at world 1)
    gives the same loss, NaN flag and training state as the separate finish launch."""
    ctx = DistContext(device=cuda)
    base = dict(batch=32, data_len=800, use_quantumnat=True, hip_graphs=False)
    a = FlagshipTrainer(FlagshipConfig(**base), ctx)
    b = FlagshipTrainer(FlagshipConfig(**base), ctx)
    b.hstep.defer_loss = False
    for _ in range(3):
        a.step()
        b.step()
        torch.cuda.synchronize()
        assert a.hstep.nmse.pending_finish is None
        assert torch.equal(a.hloss, b.hloss) and torch.equal(a.skip_flags(), b.skip_flags())
    for x, y in zip(_all_state(a), _all_state(b)):
        assert torch.equal(x, y)


def test_update_kernel_writes_the_conv_weight_images(cuda):
    """The HDCE Adam launch writes the conv weights' forward / dgrad B-fragment images (PackScatter)
    and advances the batch cursor: the images equal a fresh pack_weights of the updated weights."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    ctx = DistContext(device=cuda)
    tr = FlagshipTrainer(FlagshipConfig(batch=32, data_len=800, hip_graphs=False), ctx)
    assert tr._adam_pack() is not None
    conv = tr.hstep.conv
    for i in range(3):
        tr.step()
    torch.cuda.synchronize()
    assert int(tr.cur[0, 0]) == 3 * tr.B
    got = [t.clone() for t in conv.wpk] + [t.clone() for t in conv.wpk_t if t is not None]
    conv.pack_weights(nat.stream_ptr(cuda))
    torch.cuda.synchronize()
    ref = list(conv.wpk) + [t for t in conv.wpk_t if t is not None]
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("graphs", [False, True])
def test_fused_fc_adam_matches_separate_adam(cuda, graphs):
    """The FC weight's Adam step inside the weight-gradient GEMM's epilogue (dW never written) == the separate
    gradient GEMM + Adam launch BIT FOR BIT over 4 steps (both apply common.h adam_elem): weights, moments,
    bf16 shadow, step counters; and a NaN loss skips the fused update too."""
    ctx = DistContext(device=cuda)
    base = dict(batch=64, data_len=800, use_quantumnat=False, hip_graphs=graphs)
    ref = FlagshipTrainer(FlagshipConfig(fused_fc_adam=False, **base), ctx)
    fus = FlagshipTrainer(FlagshipConfig(fused_fc_adam=True, **base), ctx)
    assert fus.fused_adam and not ref.fused_adam
    ref.run(4)
    fus.run(4)
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(_all_state(ref), _all_state(fus))):
        assert torch.equal(a, b), (i, float((a.float() - b.float()).abs().max()))
    assert bool((fus.hopt.step_t == 4.0).all()), fus.hopt.step_t
    before = [t.clone() for t in _all_state(fus)[:7]]   # (weights, moments, shadow: not the BN statistics)
    fus.store.Yp.fill_(float("nan"))
    fus.run(1)
    torch.cuda.synchronize()
    assert float(fus.hskip) != 0.0
    for i, (a, b) in enumerate(zip(before, _all_state(fus)[:7])):
        assert torch.equal(a, b), i   # (the whole HDCE step skipped, the fused FC update included)


@pytest.mark.parametrize("mode", ["indep", "serial"])
def test_slab_fed_adam_matches_slab_launch(cuda, monkeypatch, mode):
    """The HDCE update summing the step's gradient slabs itself (knobs.KNOBS.adam_slabs: optim.hip AdamSlabs -- conv
    weights, BN, FC bias) == the slab-reduction launch before a plain update, bit for bit over 6 steps: the same row
    order per column and the same combine as conv.hip's slab_rows_sum4_body."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS
    ctx = DistContext(device=cuda)
    base = dict(batch=32, data_len=800, use_quantumnat=True, qsc_grid_bwd=128, stream_mode=mode,
                hip_graphs=mode != "serial")
    trs = []
    for on in (False, True):
        monkeypatch.setattr(KNOBS, "adam_slabs", on)
        tr = FlagshipTrainer(FlagshipConfig(steps_per_graph=3, **base), ctx)
        assert tr.adam_slabs == on
        tr.run(6)
        torch.cuda.synchronize()
        trs.append(tr)
    for i, (a, b) in enumerate(zip(_all_state(trs[0]), _all_state(trs[1]))):
        assert torch.equal(a, b), (i, float((a.float() - b.float()).abs().max()))
    assert torch.equal(trs[0].hloss, trs[1].hloss)


def test_dropped_trainer_then_new_capture_and_replay(cuda):
    """Graph lifetime in the product code: a trainer dropped right after run() -- no sync, its
    replays possibly still on the device -- parks its graph executables (GraphedStep.__del__ makes no HIP call:
    a collection can run inside another graph's capture or replay; they are destroyed at exit), so another
    trainer can capture and replay at once.  Also the explicit close() bench.py's plan selection uses.
    (tests/conftest.py no longer synchronises / collects between tests.)"""
    import gc
    ctx = DistContext(device=cuda)
    cfg = FlagshipConfig(batch=32, data_len=400, steps_per_graph=3)
    a = FlagshipTrainer(cfg, ctx)
    a.run(7)                       # (graph sets 1, 3 and a merged tail; nothing synchronised after the replays)
    del a
    gc.collect()                   # (the trainer <-> graph-set cycle goes here, with replays maybe in flight)
    b = FlagshipTrainer(cfg, ctx)
    b.run(5)
    c = FlagshipTrainer(cfg, ctx)
    c.run(4)
    b.close()                      # (explicit release while c's graphs stay alive)
    c.run(4)
    torch.cuda.synchronize()
    assert torch.isfinite(c.hloss).all() and torch.isfinite(c.qloss).all()
    with pytest.raises(RuntimeError):
        b.run(1)                   # (a closed trainer cannot step)
    c.close()
