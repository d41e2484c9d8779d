import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# on a GPU box: the native crash report (csrc/hip/runtime.hip crash_handler) also goes to a file that outlives
# pytest's capture of fd 2 (a host fault kills the process before the captured output is shown)
if os.environ.get("GRAFT_REPO_ROOT") and "QDML_CRASH_LOG" not in os.environ:
    _out = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out")
    os.makedirs(_out, exist_ok=True)
    os.environ["QDML_CRASH_LOG"] = os.path.join(_out, "native_crash.log")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU tests")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    nat.hip_lib()  # must load: GPU tests never fall back silently
    return torch.device("cuda", 0)
