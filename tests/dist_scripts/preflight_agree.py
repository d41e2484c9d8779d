"""Every rank runs the RCCL capture pre-flight; they must agree (on a CPU box: False on every rank).

    preflight_agree.py OUT"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.capture_probe import (  # noqa: E402
    preflight)

if __name__ == "__main__":
    ok = preflight(timeout=60)
    with open(f"{sys.argv[1]}.{os.environ['RANK']}", "w") as f:
        f.write(f"{int(ok)}\n")
