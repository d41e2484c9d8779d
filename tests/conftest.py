import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


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


@pytest.fixture(autouse=True)
def _gpu_teardown(request):
    """After each GPU test: finish its work and collect its graphs / trainers now, so their HIP graph executables
    and memory pools are released between tests -- not by a garbage collection that happens to run inside the next
    test's capture or replay."""
    yield
    if "cuda" in request.fixturenames:
        import gc

        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            gc.collect()
            torch.cuda.synchronize()
