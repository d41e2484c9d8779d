"""Communicator plumbing that needs no GPU: the RCCL binding (torch's librccl, one per process), and the
capture guard -- a graph capture must not begin while a gradient collective is still pending (round 3's
captured-collective abort, docs/CONCURRENCY.md "captured collectives")."""
import os

import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel import comm
from quantum_distributed_machine_learning_ris_channel_estimation_amd.utils.profiling import GraphedStep


def test_rccl_binds_torchs_library():
    assert comm.rccl_path().endswith("librccl.so") or "librccl" in comm.rccl_path()
    v = comm.rccl_version()
    assert v >= 22000, v            # (NCCL API 2.20+)
    uid = comm.new_unique_id()
    assert len(uid) == 128 and uid != comm.new_unique_id()


def test_rccl_rejects_host_tensors():
    c = comm.RcclComm.__new__(comm.RcclComm)
    with pytest.raises(comm.CommError):
        c._dt(torch.zeros(4))


def test_pre_capture_runs_guards_and_refuses_pending_collectives():
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext, GradBuckets
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        ctx = DistContext(world=1, backend="gloo", forced=True)
        g = torch.ones(8)
        bk = GradBuckets(ctx, {"a": [g]})
        gs = GraphedStep(lambda: None, enabled=False, guards=(bk.assert_quiescent,))
        gs.pre_capture()                      # nothing pending
        bk.launch("a")
        with pytest.raises(RuntimeError, match="pending"):
            gs.pre_capture()
        bk.wait()
        gs.pre_capture()
        assert torch.equal(g, torch.ones(8))
    finally:
        dist.destroy_process_group()
