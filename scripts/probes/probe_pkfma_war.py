#!/usr/bin/env python3
"""Round 6: the root-cause probe for the QSC preprocess forward's lanes-48..63 misread (docs/CONCURRENCY.md).

Runs csrc/hip/runtime.hip qd_pkfma_war_probe in every mode and prints, per mode, the (iteration, wave) events where a
packed-FP32 FMA's result was not wave-uniform although every lane read the same LDS address -- i.e. some lanes read
the registers AFTER the younger ds_read_b64 had overwritten them -- and the OR of the lane masks of those events.

    python scripts/probes/probe_pkfma_war.py [iters] [grid]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat  # noqa: E402

MODES = [(0, "v_pk_fma_f32, idle partners"), (1, "v_pk_fma_f32, MFMA partners"),
         (1 | 4, "v_pk_fma_f32, MFMA partners, 8-cycle pad"), (1 | 8, "v_pk_fma_f32, MFMA partners, 24-cycle pad"),
         (2, "2 x v_fma_f32, idle partners"), (2 | 1, "2 x v_fma_f32, MFMA partners")]


def run(mode: int, iters: int, grid: int):
    f = nat.fn(nat.hip_lib(), "qd_pkfma_war_probe", [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p])
    out = torch.zeros(132, dtype=torch.int32, device="cuda")
    nat.check(f(mode, iters, grid, nat.ptr(out), nat.stream_ptr(out.device)), "pkfma_war_probe")
    torch.cuda.synchronize()
    ev, n, _, mask = [int(v) & 0xffffffff for v in out[:4].tolist()]
    lanes = out[4:].view(torch.float32).view(64, 2).cpu()
    return ev, n, mask, lanes


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    grid = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    print(f"iters {iters} per probe wave, grid {grid} x (4 probe + 4 partner waves)")
    for mode, name in MODES:
        ev, n, mask, vals = run(mode, iters, grid)
        lanes = [i for i in range(32) if mask >> i & 1]
        print(f"mode {mode:2d} {name:46s} events {ev:8d} / {n:9d}  lanes (mod 32) {lanes}", flush=True)
        if ev:
            print("   wave 0, iteration 0, acc (x, y) of lanes 0 / 15 / 16 / 31 / 32 / 47 / 48 / 63:",
                  [tuple(round(float(v), 6) for v in vals[i]) for i in (0, 15, 16, 31, 32, 47, 48, 63)], flush=True)


if __name__ == "__main__":
    main()
