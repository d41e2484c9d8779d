#!/usr/bin/env python3
"""Pick the fastest hipBLASLt / rocBLAS solution for every library GEMM of the flagship step
(PyTorch TunableOp) and store the choices in-tree, so runs replay them without tuning.

    python scripts/tune_gemm.py [--out quantum_.../tuning/tunableop_gfx950.csv] [--qubits 8]

The FC_P128 GEMMs (M = 2304 rows, N = 2048, K = 4096: forward, data gradient, weight gradient)
are plain library GEMMs; TunableOp times every solution the libraries offer for each shape and
keeps the fastest (the default heuristic pick is measured alongside, see the printed table).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train import flagship as fl
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext

    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=fl.TUNABLEOP_FILE)
    ap.add_argument("--qubits", type=int, default=8)
    ap.add_argument("--pilot", type=int, default=128)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_iterations(a.iters)
    tun.set_filename(a.out, insert_device_ordinal=False)
    ctx = DistContext(device=torch.device("cuda", 0))
    torch.cuda.set_device(0)
    cfg = fl.FlagshipConfig(pilot_num=a.pilot, n_qubits=a.qubits, dtype=a.dtype, hip_graphs=False,
                            stream_mode="serial", tunableop=False)
    tr = fl.FlagshipTrainer(cfg, ctx)
    t0 = time.time()
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    if hasattr(tun, "write_file"):
        tun.write_file()
    print(f"tuned in {time.time() - t0:.1f} s -> {a.out} (TunableOp also writes it at exit)")
    for r in tun.get_results():
        print(r)


if __name__ == "__main__":
    main()
