"""Debug: a multi-stream plan (default dagi: independent HDCE / QSC chains) vs serial eager, step by
step, over several fresh trainer pairs; reports the first step whose QSC weights differ.

    PYTHONPATH=. python scripts/dbg_dagi.py [mode] [trials]

(This found that capturing the dagi QSC chain AFTER the HDCE chain gives wrong QSC results on the
ROCm 7.x graph executor; see FlagshipTrainer._indep_body.)"""
import sys

import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import FlagshipConfig, FlagshipTrainer


def main():
    ctx = DistContext(device=torch.device("cuda", 0))
    base = dict(batch=32, data_len=800, use_quantumnat=True, qsc_grid_bwd=128)
    mode = sys.argv[1] if len(sys.argv) > 1 else "dagi"
    bad = 0
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    for trial in range(int(sys.argv[2]) if len(sys.argv) > 2 else 5):
        ref = FlagshipTrainer(FlagshipConfig(hip_graphs=False, stream_mode="serial", **base), ctx)
        dag = FlagshipTrainer(FlagshipConfig(hip_graphs=True, stream_mode=mode.replace("graphs", ""), steps_per_graph=k,
                                             **base), ctx)   # (mode "serialgraphs": one-stream graphs)
        dag.capture(preserve=True, k=k)
        first = None
        for s in range(4):
            for _ in range(k):
                ref.step()
            dag.run(k)
            torch.cuda.synchronize()
            dq = float((ref.qspace.flat - dag.qspace.flat).abs().max())
            dh = float((ref.hdce.space.flat - dag.hdce.space.flat).abs().max())
            if dq > 0 and first is None:
                d = (ref.qspace.flat - dag.qspace.flat).abs()
                per = {n: float(d[o:o + p.numel()].max()) for n, o, p in
                       zip(dag.qspace.names, dag.qspace.offsets, dag.qspace.params)}
                gm = {n: float((ref.qspace.grad - dag.qspace.grad)[o:o + p.numel()].abs().max()) for n, o, p in
                      zip(dag.qspace.names, dag.qspace.offsets, dag.qspace.params)}
                print("  per-param max |dw|", per, flush=True)
                print("  per-param max |dgrad| (last step)", gm, flush=True)
                print("  step_t", ref.qopt.step_t.tolist(), dag.qopt.step_t.tolist(), "m diff",
                      float((ref.qopt.m - dag.qopt.m).abs().max()), flush=True)
            if (dq > 0 or dh > 0) and first is None:
                first = (s, "q", dq, "h", dh, float(ref.qloss), float(dag.qloss), float(ref.hloss[0]), float(dag.hloss[0]),
                         ref.cur[:, 0].tolist(), dag.cur[:, 0].tolist(), int(ref.cstep.hip.noise_ctr), int(dag.cstep.hip.noise_ctr))
        bad += first is not None
        print(mode, "trial", trial,
              "first mismatch", first, flush=True)
    print("SUMMARY", mode, "k", k, "bad", bad)


if __name__ == "__main__":
    main()
