"""Debug: which buffer of the QSC chain first differs between a multi-stream graph plan and the serial
eager run?  Compares, after every replay, the QSC step's intermediates in chain order (gather output,
noisy weights, preprocess outputs, angles, expectation values, head gradients, adjoint outputs,
slabs, gradient, moments, weights).

    PYTHONPATH=. python scripts/dbg_bisect.py [mode] [steps_per_graph] [replays] [trials]
"""
import sys

import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import FlagshipConfig, FlagshipTrainer

CHAIN = ["xq", "wnoisy", "p2", "p1s", "c1", "c2", "angles", "psave", "E", "loss", "dE", "dang", "dpre", "preslab",
         "qslab", "grad", "m", "v", "flat"]


def bufs(tr):
    h = tr.cstep.hip
    out = {"xq": tr.gat.xq}
    for n in CHAIN:
        t = getattr(h, n, None)
        if isinstance(t, torch.Tensor):
            out[n] = t
    out.update(grad=tr.qspace.grad, m=tr.qopt.m, v=tr.qopt.v, flat=tr.qspace.flat)
    return out


def dep_gap():
    """(QD_DEPSTAMP builds) min(qsim_fwd start) - max(qsc2_fwd end) of the last step, microseconds."""
    import ctypes
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    lib = nat.hip_lib()
    if not hasattr(lib, "qd_dep_fwd_end"):
        return None
    a, b = (ctypes.c_ulonglong * 8192)(), (ctypes.c_ulonglong * 8192)()
    na, nb = ctypes.c_int(), ctypes.c_int()
    lib.qd_dep_fwd_end(a, ctypes.byref(na))
    lib.qd_dep_qsim_start(b, ctypes.byref(nb))
    end = max(a[:na.value])
    start = min(b[:nb.value])
    return (int(start) - int(end)) * 0.01


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "qsc"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    reps = min(reps, 16 // k)   # (720 samples per stream at batch 32: more steps wrap the epoch, and the two
    #                             trainers then draw different permutations)
    trials = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    ctx = DistContext(device=torch.device("cuda", 0))
    base = dict(batch=32, data_len=800, use_quantumnat=True, qsc_grid_bwd=128)
    nbad = 0
    for trial in range(trials):
        ref = FlagshipTrainer(FlagshipConfig(hip_graphs=False, stream_mode="serial", **base), ctx)
        # mode "split": the data-parallel execution plan (5 graphs, FC Adam on its own stream) at world 1
        kw = dict(stream_mode="dagq", split_graphs=True) if mode == "split" else dict(stream_mode=mode, steps_per_graph=k)
        dag = FlagshipTrainer(FlagshipConfig(hip_graphs=True, **kw, **base), ctx)
        dag.capture(preserve=True, k=1 if mode == "split" else k)
        first = None
        for r in range(reps):
            for _ in range(k):
                ref.step()
            dag.run(k)
            torch.cuda.synchronize()
            gap = dep_gap()
            if gap is not None:
                print(f"trial {trial} replay {r}: qsim_fwd start - qsc2_fwd end = {gap:.2f} us", flush=True)
            a, b = bufs(ref), bufs(dag)
            diff = []
            for n in CHAIN:
                if n in a and n in b and a[n].shape == b[n].shape and not torch.equal(a[n], b[n]):
                    d = (a[n].float() - b[n].float()).abs()
                    idx = (a[n] != b[n]).nonzero()
                    diff.append((n, float(d.max()), int(idx.shape[0]), a[n].numel(), idx[0].tolist(), idx[-1].tolist()))
            if diff and gap is not None:   # what did the dag's forward actually read?
                import ctypes
                from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
                xs = (ctypes.c_float * (8192 * 9))()
                nat.hip_lib().qd_dep_xseen(xs)
                B = dag.cstep.hip.angles.shape[0]
                seen = torch.tensor(xs[:B * 9]).view(B, 9)
                ang = b["angles"].cpu()
                wn = b["wnoisy"].cpu().view(-1, 48).sum(1)
                grp = B // wn.numel()
                bad_x = (seen[:, :8] != ang).any(1).nonzero().flatten().tolist()
                bad_w = ((seen[:, 8] - wn.repeat_interleave(grp)).abs() > 1e-4).nonzero().flatten().tolist()
                print(f"   forward read stale angles for samples {bad_x}, weights (sum) differ for {bad_w[:12]}", flush=True)
                if bad_x:
                    i = bad_x[0]
                    print("   seen", seen[i, :8].tolist(), "final", ang[i].tolist(), flush=True)
            if diff:
                print(f"trial {trial} replay {r}: first differing buffer {diff[0]}", flush=True)
                print("   all:", [(x[0], x[2]) for x in diff], flush=True)
                first = first or (r, diff[0][0])
                break
        nbad += first is not None
        print(f"trial {trial} first {first}", flush=True)
    print("SUMMARY", mode, "k", k, "bad", nbad, "of", trials)


if __name__ == "__main__":
    main()
