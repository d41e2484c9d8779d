"""Structured metrics (rank-0 JSONL) and throughput meters.

Reference logging is ``print`` only: per-epoch LR + timestamp (R:171-173),
per-50-iteration loss (R:206-208), val NMSE (R:268-270), QSC loss/accuracy (R:375, R:414).
We keep those human-readable lines and add a machine-readable JSONL stream with
epoch, step, loss, accuracy, NMSE (linear and dB), LR, samples/sec and world size.
"""
from __future__ import annotations

import json
import math
import os
import time
from typing import Any, Dict, Optional


def to_db(x: float) -> float:
    return 10.0 * math.log10(x) if x > 0 else float("-inf")


class MetricsLogger:
    def __init__(self, path: Optional[str], rank: int = 0, world: int = 1, run: str = "train"):
        self.path = path if rank == 0 else None
        self.world = world
        self.run = run
        if self.path:
            d = os.path.dirname(self.path)
            if d:
                os.makedirs(d, exist_ok=True)

    def log(self, **rec: Any) -> None:
        if not self.path:
            return
        rec = {"ts": time.time(), "run": self.run, "world_size": self.world, **rec}
        with open(self.path, "a") as f:
            f.write(json.dumps(rec, default=_default) + "\n")


def _default(o):
    try:
        return float(o)
    except Exception:
        return str(o)


class Throughput:
    """samples/sec over an interval; call ``mark(samples)`` after a synchronising point."""

    def __init__(self):
        self.t0 = time.perf_counter()
        self.samples = 0

    def add(self, n: int) -> None:
        self.samples += n

    def rate(self, reset: bool = True) -> float:
        t = time.perf_counter()
        r = self.samples / max(t - self.t0, 1e-9)
        if reset:
            self.t0, self.samples = t, 0
        return r
