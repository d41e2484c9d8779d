"""One-process-per-GPU launcher (torchrun-compatible environment contract).

Reference: the only multi-GPU launch in the reference is setting
``CUDA_VISIBLE_DEVICES="0,1,2,3"`` in-process before ``DataParallel`` (R:135-137, R:308-310).
Here every rank is its own process with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT set, so ``torch.distributed.run`` and this launcher are interchangeable.  If
any rank fails, the others are terminated and the launcher exits with that rank's code.

    python -m quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.launch \
        --nproc 8 -- python bench.py --gpus 8
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def launch(cmd: List[str], nproc: int, master_addr: str = "127.0.0.1", master_port: Optional[int] = None,
           extra_env: Optional[dict] = None, poll_s: float = 0.2) -> int:
    port = master_port or free_port(master_addr)
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update(extra_env or {})
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nproc), "LOCAL_WORLD_SIZE": str(nproc),
                    "MASTER_ADDR": master_addr, "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    rc = 0
    try:
        alive = list(range(nproc))
        while alive:
            for r in list(alive):
                code = procs[r].poll()
                if code is None:
                    continue
                alive.remove(r)
                if code != 0 and rc == 0:
                    rc = code
                    for q in alive:  # fail fast: stop the remaining ranks (their own process groups only)
                        try:
                            os.killpg(procs[q].pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        rc = 130
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--nproc", type=int, required=True)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing command")
    return launch(cmd, a.nproc, a.master_addr, a.master_port)


if __name__ == "__main__":
    sys.exit(main())
