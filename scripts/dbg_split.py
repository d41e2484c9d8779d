"""Debug helper: a graphed multi-stream FlagshipTrainer vs the serial eager one, step by step."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)

cuda = torch.device("cuda", 0)
ctx = DistContext(device=cuda)
base = dict(batch=32, data_len=800, use_quantumnat=True)
cases = [(m, int(k), s == "1") for m, k, s in (a.split(":") for a in sys.argv[1:])] or [("qsc", 2, False)]
for mode, k, split in cases:
    ref = FlagshipTrainer(FlagshipConfig(hip_graphs=False, stream_mode="serial", **base), ctx)
    dag = FlagshipTrainer(FlagshipConfig(hip_graphs=True, stream_mode=mode, split_graphs=split, steps_per_graph=k,
                                         **base), ctx)
    dag.capture(preserve=True, k=k)
    nohdce = __import__("os").environ.get("QDML_DBG_QSC") == "nohdce"
    for rep in range(3):
        for _ in range(k):
            if nohdce:   # the reference runs only the QSC part too
                ref._gather()
                ref._qsc_branch(with_opt=True)
                ref.cursor += ref.B
            else:
                ref.step()
        dag.run(k)
        torch.cuda.synchronize()
        d = [(n, float((p.detach() - dag.qspace.params[i].detach()).abs().max()))
             for i, (n, p) in enumerate(zip(ref.qspace.names, ref.qspace.params))]
        print(mode, k, split, "replay", rep, "qsc param diff", [x for x in d if x[1] > 0],
              "hdce diff", float((ref.hdce.space.flat - dag.hdce.space.flat).abs().max()),
              "loss", float(ref.qloss), float(dag.qloss), "noise ctr", int(ref.cstep.hip.noise_ctr),
              int(dag.cstep.hip.noise_ctr), "cur", ref.cur[:, 0].tolist(), dag.cur[:, 0].tolist(), flush=True)
