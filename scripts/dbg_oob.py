"""Debug: does one half of the flagship step (HDCE or QSC) write into a buffer owned by the other?

A stray write that lands in memory the other chain rewrites before reading is harmless when the
chains run one after the other and corrupts it when they overlap -- the signature of the multi-stream
drift (FlagshipTrainer: dagi / qsc modes).  Every persistent tensor reachable from the trainer is
classified by owner (HDCE side / QSC side); each half runs ALONE (eager, one stream) and every
tensor of the other side is compared bitwise before / after.  Also fills the gaps between
allocations?  No -- only tensors the trainer owns are checked; run with PYTORCH_NO_HIP_MEMORY_CACHING=1
to give every tensor its own allocation.

    PYTHONPATH=. python scripts/dbg_oob.py
"""
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import FlagshipConfig, FlagshipTrainer


def tensors(root, depth=4, seen=None, path="", out=None):
    """(path, tensor) for every CUDA tensor reachable through attributes / lists / dicts."""
    seen = set() if seen is None else seen
    out = [] if out is None else out
    if id(root) in seen or depth < 0:
        return out
    seen.add(id(root))
    if isinstance(root, torch.Tensor):
        if root.is_cuda:
            out.append((path, root))
        return out
    if isinstance(root, torch.nn.Module):
        for n, p in list(root.named_parameters()) + list(root.named_buffers()):
            tensors(p, depth - 1, seen, f"{path}.{n}", out)
    items = []
    if isinstance(root, dict):
        items = list(root.items())
    elif isinstance(root, (list, tuple)):
        items = list(enumerate(root))
    elif hasattr(root, "__dict__") and type(root).__module__.startswith(("quantum_distributed", "__main__")):
        items = list(vars(root).items())
    for k, v in items:
        if isinstance(v, (torch.Tensor, dict, list, tuple, torch.nn.Module)) or hasattr(v, "__dict__"):
            tensors(v, depth - 1, seen, f"{path}.{k}", out)
    return out


def spans(ts):
    """unique (ptr, nbytes, path, tensor) by storage span"""
    res = {}
    for p, t in ts:
        st = t.untyped_storage()
        key = (st.data_ptr(), st.nbytes())
        if key not in res:
            res[key] = (p, t)
    return res


def main():
    ctx = DistContext(device=torch.device("cuda", 0))
    tr = FlagshipTrainer(FlagshipConfig(hip_graphs=False, stream_mode="serial", batch=256), ctx)
    tr.step()
    torch.cuda.synchronize()
    q_roots = {"cstep": tr.cstep, "qspace": tr.qspace, "qopt": tr.qopt, "qsc": tr.qsc, "qslabs": tr.qslabs}
    h_roots = {"hstep": tr.hstep, "hdce": tr.hdce, "hopt": tr.hopt, "gat_x1": tr.gat.x1, "gat_rowoff": tr.gat.rowoff,
               "gat_rowden": tr.gat.rowden}
    q = spans([x for k, r in q_roots.items() for x in tensors(r, path=k)])
    h = spans([x for k, r in h_roots.items() for x in tensors(r, path=k)])
    shared = set(q) & set(h)
    print("QSC spans", len(q), "HDCE spans", len(h), "shared", [q[k][0] for k in shared], flush=True)
    # every storage of both sides as raw bytes, by address (to report neighbours)
    allspans = sorted([(k[0], k[1], "Q " + v[0]) for k, v in q.items()] + [(k[0], k[1], "H " + v[0]) for k, v in h.items()])

    def snap(side):
        return {k: torch.frombuffer(bytearray(0), dtype=torch.uint8) if k[1] == 0 else
                torch.empty(0, dtype=torch.uint8, device="cuda").set_(v[1].untyped_storage(), 0, (k[1],)).clone()
                for k, v in side.items() if k not in shared}

    def compare(before, side, label):
        bad = []
        for k, b in before.items():
            a = torch.empty(0, dtype=torch.uint8, device="cuda").set_(side[k][1].untyped_storage(), 0, (k[1],))
            if not torch.equal(a, b):
                idx = (a != b).nonzero().flatten()
                bad.append((side[k][0], hex(k[0]), k[1], int(idx[0]), int(idx[-1]), int(idx.numel())))
        print(label, "changed:", bad if bad else "none", flush=True)
        return bad

    # HDCE half alone: must not touch any QSC-side byte
    for rep in range(3):
        b = snap(q)
        tr.next_batch()
        tr._gather(hdce=True, classifier=False)
        tr._hdce_graph()
        torch.cuda.synchronize()
        bad = compare(b, q, f"[rep {rep}] HDCE half -> QSC-side buffers")
        # QSC half alone: must not touch any HDCE-side byte (x1 / rowoff are gather outputs it does not write)
        b = snap(h)
        tr._gather(hdce=False, classifier=True)
        tr._qsc_branch(with_opt=True)
        torch.cuda.synchronize()
        bad2 = compare(b, h, f"[rep {rep}] QSC half -> HDCE-side buffers")
        for lst in (bad, bad2):
            for name, ptr, nb, i0, i1, n in lst:
                a = int(ptr, 16)
                near = [(hex(s), n_, nm) for s, n_, nm in allspans if s + n_ >= a - 65536 and s <= a + nb + 65536]
                print("  neighbours of", name, near, flush=True)
    print("DONE")


if __name__ == "__main__":
    main()
