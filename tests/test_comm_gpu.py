"""The framework's own RCCL communicator (parallel/comm.py over csrc/hip/comm.hip) on the GPU: every
collective eager and captured in a HIP graph at world 1 (QDML_FORCE_DIST=1), and a runner HDCE run whose
graphed steps capture the bucketed gradient all-reduces == the same run eager, bit for bit."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_rccl_collectives_and_captured_runner_world1(tmp_path):
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch import launch
    here = os.path.dirname(os.path.abspath(__file__))
    out = str(tmp_path / "rc")
    rc = launch([sys.executable, os.path.join(here, "dist_scripts", "rccl_world1.py"), out, str(tmp_path / "ws")],
                nproc=1, extra_env={"OMP_NUM_THREADS": "2", "QDML_FORCE_DIST": "1"})
    assert rc == 0
    rec = open(f"{out}.0").read().split()
    assert rec[0] == "1", rec
