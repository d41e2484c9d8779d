#!/usr/bin/env python3
"""Round 5: the fp8 estimator's forward GEMM with the loss in its epilogue (gemm.hip EPI_NMSE, qd_gemm_fwd_nmse_f8)
against the same e4m3 GEMM without it (qd_gemm_fwd_f8), at the flagship shape, from one real flagship step's buffers.
Run under rocprofv3 --kernel-trace --stats: the kernels' own durations are the measurement.

    python scripts/probes/probe_nmse_epi.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.fc import gemm_fwd_f8  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import (  # noqa: E402
    FlagshipConfig, FlagshipTrainer)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda")
    ctx = DistContext(device=dev)
    tr = FlagshipTrainer(FlagshipConfig(batch=256, data_len=1600, hip_graphs=False, use_quantumnat=False,
                                        stream_mode="serial", dtype="fp8"), ctx)
    nm = tr.hstep.nmse
    seen = {}
    orig = nm.gemm_fused

    def spy(*a, **k):
        seen["args"], seen["kw"] = a, k
        return orig(*a, **k)

    nm.gemm_fused = spy
    tr.next_batch()
    tr._dp_g1()
    tr._dp_g2()
    torch.cuda.synchronize()
    nm.gemm_fused = orig
    a, k = seen["args"], dict(seen["kw"])
    k["bias_slabs"], k["defer_loss"] = None, False   # (the loss finish and bias reduction as launches of their own)
    A, W = a[0], a[1]
    Y = torch.empty(A.shape[0], W.shape[0], device=dev, dtype=torch.bfloat16)
    for _ in range(reps):
        orig(*a, **k)
        gemm_fwd_f8(A, W, k["deq"], None, out=Y, cfg=2)
    torch.cuda.synchronize()
    print("done", A.shape, W.shape, flush=True)


if __name__ == "__main__":
    main()
