#!/usr/bin/env python3
"""Round 5 diagnosis: test_multistream_graph_matches_serial_eager fails for the split-forward plans (qsc_start="conv",
fc_adam_next) only with the fused-loss forward (KNOBS.hand_gemm "fwd").  Step the serial eager reference and the
graph plan (k = 1 graph, one step per replay) side by side and print, per step, where they first differ: the QSC
loss, QSC gradient, QSC weights, QSC optimizer moments, skip flags, HDCE loss / weights.

    python scripts/probes/probe_split_fused.py [fwd|fwdplain] [conv|fcnext] [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd.knobs import KNOBS  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


def d(a, b):
    return float((a.float() - b.float()).abs().max())


def main():
    hg = sys.argv[1] if len(sys.argv) > 1 else "fwd"
    mode = sys.argv[2] if len(sys.argv) > 2 else "fcnext"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    KNOBS.hand_gemm = hg + ",wgrad,dgrad"
    dev = torch.device("cuda")
    if os.environ.get("PROBE_LDS_POISON"):   # every launch preceded by an LDS fill (_native.set_lds_poison)
        import quantum_distributed_machine_learning_ris_channel_estimation_amd._native as nat0
        nat0.set_lds_poison(int(os.environ["PROBE_LDS_POISON"], 16))
    ctx = DistContext(device=dev)
    base = dict(batch=32, data_len=800, use_quantumnat=True, qsc_grid_bwd=128)
    opts = {"conv": {"qsc_start": "conv"}, "fcnext": {"fc_adam_next": 256}}[mode]
    ref = FlagshipTrainer(FlagshipConfig(hip_graphs=False, stream_mode="serial", **base), ctx)
    dag = FlagshipTrainer(FlagshipConfig(hip_graphs=True, stream_mode="indep", steps_per_graph=1, **opts, **base), ctx)
    dag.capture(preserve=True, k=1)
    torch.cuda.synchronize()
    # every device buffer of the two chains: do any two of them share memory?
    bufs = []

    def collect(prefix, obj, depth=0):
        for name, t in list(vars(obj).items()):
            if isinstance(t, torch.Tensor) and t.is_cuda and t.numel() > 0:
                bufs.append((f"{prefix}.{name}", t.data_ptr(), t.numel() * t.element_size()))
            elif isinstance(t, tuple) and depth == 0:
                for i, u in enumerate(t):
                    if isinstance(u, torch.Tensor) and u.is_cuda and u.numel() > 0:
                        bufs.append((f"{prefix}.{name}[{i}]", u.data_ptr(), u.numel() * u.element_size()))
    for pre, o in (("gat", dag.gat), ("hstep", dag.hstep), ("nmse", dag.hstep.nmse), ("conv", dag.hstep.conv),
                   ("cstep", dag.cstep), ("qhip", dag.cstep.hip), ("dag", dag), ("qspace", dag.qspace),
                   ("hspace", dag.hdce.space), ("qopt", dag.qopt), ("hopt", dag.hopt), ("hdce", dag.hdce)):
        if o is not None:
            collect(pre, o)
    for pre, o in (("conv", dag.hstep.conv),):
        for name, t in vars(o).items():
            if isinstance(t, (list, tuple)):
                for i, u in enumerate(t):
                    if isinstance(u, torch.Tensor) and u.is_cuda and u.numel() > 0:
                        bufs.append((f"{pre}.{name}[{i}]", u.data_ptr(), u.numel() * u.element_size()))
    bufs.sort(key=lambda b: b[1])
    seen = set()
    for i in range(len(bufs)):
        for j in range(i + 1, len(bufs)):
            a, b = bufs[i], bufs[j]
            if b[1] >= a[1] + a[2]:
                break
            if a[1] == b[1] and a[2] == b[2]:
                continue   # (the same tensor under two names)
            key = (a[0], b[0])
            if key not in seen:
                seen.add(key)
                print(f"OVERLAP {a[0]} [{a[1]:#x}, +{a[2]}) with {b[0]} [{b[1]:#x}, +{b[2]})", flush=True)
    print(f"{len(bufs)} buffers checked", flush=True)
    if os.environ.get("PROBE_MAP"):
        for name, ptr, nb in bufs:
            print(f"MAP {ptr:#x} {nb:>10d} {name}", flush=True)
    print(f"[{hg} {mode}] after capture: qflat {d(ref.qspace.flat, dag.qspace.flat):.3e} hflat "
          f"{d(ref.hdce.space.flat, dag.hdce.space.flat[:ref.hdce.space.flat.numel()]):.3e} noise "
          f"{int(ref.cstep.hip.noise_ctr.flatten()[0]) if ref.cstep.hip is not None else -1} / "
          f"{int(dag.cstep.hip.noise_ctr.flatten()[0]) if dag.cstep.hip is not None else -1}", flush=True)
    poison = os.environ.get("PROBE_POISON_XQ") == "1"
    recompute = os.environ.get("PROBE_RECOMPUTE") == "1"
    for s in range(steps):
        pre = (ref.qspace.flat.clone(), dag.qspace.flat.clone())
        ref.step()
        if poison:   # a QSC forward that reads xq before this step's QSC gather wrote it would see NaN
            dag.gat.xq.fill_(float("nan"))
        dag.run(1)
        torch.cuda.synchronize()
        print(f"step {s + 1}: qloss {float(ref.qloss):.7f} / {float(dag.qloss):.7f}  hloss {float(ref.hloss[0]):.7f} / "
              f"{float(dag.hloss[0]):.7f}  qgrad {d(ref.qspace.grad, dag.qspace.grad[:ref.qspace.grad.numel()]):.3e}  "
              f"qflat {d(ref.qspace.flat, dag.qspace.flat):.3e}  qm {d(ref.qopt.m, dag.qopt.m):.3e}  "
              f"hflat {d(ref.hdce.space.flat, dag.hdce.space.flat[:ref.hdce.space.flat.numel()]):.3e}  "
              f"skip {ref.skip_flags().tolist()} / {dag.skip_flags().tolist()}  qstep {float(ref.qopt.step_t[0])} / "
              f"{dag.qopt.step_t.tolist()}  xq {d(ref.gat.xq, dag.gat.xq):.3e}", flush=True)
        if recompute and s == 0:   # the preprocess forward again, eagerly, from each side's pre-step weights
            import quantum_distributed_machine_learning_ris_channel_estimation_amd._native as nat
            for lab, tr, fl in (("ref", ref, pre[0]), ("dag", dag, pre[1])):
                h = tr.cstep.hip
                run_p1, run_ang = h.p1s.clone(), h.angles.clone()
                h._fwd_mfma(tr.gat.xq, fl, nat.stream_ptr(dev))
                torch.cuda.synchronize()
                print(f"   {lab}: eager recompute vs its step: p1s {d(run_p1, h.p1s):.3e} angles {d(run_ang, h.angles):.3e}",
                      flush=True)
                per = (run_p1 - h.p1s).abs().amax(dim=1)
                bad = torch.nonzero(per > 0).flatten().tolist()
                if bad:   # which samples, their workgroup (4 waves each) and its XCD (block % 8)
                    print(f"   {lab}: {len(bad)} of {per.numel()} samples differ; first: "
                          f"{[(b, b // 4, (b // 4) % 8) for b in bad[:24]]}", flush=True)
                    xcds = torch.tensor([(b // 4) % 8 for b in bad]).bincount(minlength=8).tolist()
                    print(f"   {lab}: differing samples per XCD of their workgroup: {xcds}", flush=True)
                    rows = torch.tensor(bad, device=dev)
                    dif = (run_p1[rows] - h.p1s[rows]).abs() > 0
                    print(f"   {lab}: per differing sample, entries that differ: {dif.sum(1).tolist()[:24]} of "
                          f"{run_p1.shape[1]}; step min p1 {float(run_p1.min()):.3e}", flush=True)
                    for b in bad[:3]:   # the differing entries (window, channel): step value / recompute value
                        ent = torch.nonzero((run_p1[b] - h.p1s[b]).abs() > 0).flatten().tolist()
                        print(f"   {lab}: sample {b}: " + ", ".join(
                            f"(w{e // 16} c{e % 16}) {float(run_p1[b, e]):.4f}/{float(h.p1s[b, e]):.4f}" for e in ent),
                            flush=True)
                    # the same forward from the POST-step weights: do the differing samples match that instead?
                    pre_p1 = h.p1s.clone()
                    h._fwd_mfma(tr.gat.xq, tr.qspace.flat, nat.stream_ptr(dev))
                    torch.cuda.synchronize()
                    per2 = (run_p1 - h.p1s).abs().amax(dim=1)
                    post_ok = [b for b in bad if float(per2[b]) == 0.0]
                    print(f"   {lab}: of the differing samples, {len(post_ok)} match a forward from the post-step "
                          f"weights; samples that differ from that one: {int((per2 > 0).sum())}", flush=True)
                    # the previous step's batch (the cursor one batch back) is not at hand; the c1 codes are
                    h.p1s.copy_(pre_p1)
        if s == 0:   # every QSC buffer of the first step: which one differs first
            for owner in ("cstep", "cstep.hip"):
                ra, da = ref, dag
                for part in owner.split("."):
                    ra, da = getattr(ra, part, None), getattr(da, part, None)
                if ra is None:
                    continue
                for name, t in sorted(vars(ra).items()):
                    u = getattr(da, name, None)
                    if isinstance(t, torch.Tensor) and isinstance(u, torch.Tensor) and t.shape == u.shape and t.is_cuda:
                        try:
                            print(f"   {owner}.{name} {tuple(t.shape)} {t.dtype}: {d(t, u):.3e}", flush=True)
                        except RuntimeError:
                            pass


if __name__ == "__main__":
    main()
