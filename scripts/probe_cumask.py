"""Does a CU-masked stream confine its kernels, and does a HIP graph replay keep the mask?

For several masks: launch the CU probe (csrc/hip/runtime.hip) eagerly on the masked stream, and
inside a captured graph replayed on that stream; count the distinct (xcc, se, sa, cu) ids seen.
"""
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops import streams as S  # noqa: E402


def run(out, stream, graph=False):
    out.zero_()
    if not graph:
        with torch.cuda.stream(stream):
            S.cu_probe_launch(out, spin=200)
        stream.synchronize()
    else:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            S.cu_probe_launch(out, spin=200)
        out.zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            g.replay()
        stream.synchronize()
    ids = S.decode(out)
    per_xcc = collections.Counter(i[0] for i in set(ids))
    return len(set(ids)), dict(sorted(per_xcc.items())), sorted(set(ids))


def main():
    dev = torch.device("cuda", 0)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(2 * 4096, dtype=torch.int32, device=dev)
    base = torch.cuda.Stream(dev)
    n, px, ids = run(out, base)
    print(json.dumps({"mask": "unmasked", "n_cu": n_cu, "distinct": n, "per_xcc": px}))
    print("first ids:", ids[:40])
    for spec in ("first:32", "first:64", "stride:8:0", "stride:4:0", "0-127", "128-255", "stride:2:1"):
        cus = S.parse_cus(spec, n_cu)
        s = S.masked_stream(cus, dev)
        got = S.stream_mask(s, n_cu)
        for graph in (False, True):
            n, px, ids = run(out, s, graph)
            print(json.dumps({"mask": spec, "n_mask": len(cus), "mask_readback_ok": got == cus,
                              "graph": graph, "distinct": n, "per_xcc": px}))
            if spec == "first:32" and not graph:
                print("ids:", ids)


if __name__ == "__main__":
    main()
