#!/usr/bin/env python3
"""Launch-configuration sweeps for the fused kernels (run on an MI355X).

Times graph-captured replays (so host launch cost drops out) of
  * QSCStepHIP (qsc_pre_fwd / qsim / head / qsim_bwd / qsc_pre_bwd) over grid sizes;
  * ConvStackHIP forward + backward over samples-per-wave / per-block knobs.
Prints one JSON line per configuration.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def time_graph(fn, iters=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def tune_qsc(n, pilot, B, grids):
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import QSC_P128
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.optim import FlatParamSpace
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.qsc import QSCStepHIP
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = QSC_P128(n_qubits=n, use_quantumnat=True, use_gradient_pruning=False, pilot_num=pilot).to(dev)
    sp = FlatParamSpace(list(m.named_parameters()), dev)
    H, W = (16, 8) if pilot == 128 else (16, 16)
    x = torch.randn(B, 2, H, W, device=dev)
    y = torch.randint(0, 3, (B,), device=dev)
    for gf, gb in grids:
        step = QSCStepHIP(m, sp, B, n_groups=9, grid_fwd=gf, grid_bwd=gb)
        us = time_graph(lambda: step(x, y))
        print(json.dumps({"op": "qsc_step", "n": n, "pilot": pilot, "B": B, "grid_fwd": gf, "grid_bwd": gb,
                          "us": round(us, 1)}), flush=True)


def tune_conv(pilot, Bs, combos):
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.conv import ConvStackHIP
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel
    dev = torch.device("cuda")
    m = HDCEModel(pilot, dev, "bf16")
    U, E = 3, 3
    for B in Bs:
        N = U * B
        x1 = torch.randn(N, 2 * E, m.H, m.W, device=dev)
        dh = torch.randn(N * E, 32 * m.H * m.W, device=dev).to(torch.bfloat16)
        for spw, spbw, spbr in combos:
            try:
                cs = ConvStackHIP(m, U, B, spw=spw, spb_w=spbw, spb_r=spbr)
                f = time_graph(lambda: cs.forward(x1, True))
                fb = time_graph(lambda: (cs.forward(x1, True), cs.backward(dh)))
            except Exception as e:  # unsupported combination
                print(json.dumps({"op": "conv", "spw": spw, "spb_w": spbw, "spb_r": spbr, "error": str(e)[:200]}))
                continue
            print(json.dumps({"op": "conv", "pilot": pilot, "B": B, "spw": spw, "spb_w": spbw, "spb_r": spbr,
                              "fwd_us": round(f, 1), "fwd_bwd_us": round(fb, 1)}), flush=True)


def tune_wgrad(pilot, B, spbs):
    """Each layer's weight-gradient launch alone, per samples-per-workgroup setting."""
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.conv import ConvStackHIP, _ptr
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel
    dev = torch.device("cuda")
    m = HDCEModel(pilot, dev, "bf16")
    U, E = 3, 3
    N = U * B
    x1 = torch.randn(N, 2 * E, m.H, m.W, device=dev)
    dh = torch.randn(N * E, 32 * m.H * m.W, device=dev).to(torch.bfloat16)
    dx = torch.randn(N, 32 * E, m.H * m.W, device=dev).to(torch.bfloat16)
    for spb in spbs:
        cs = ConvStackHIP(m, U, B, spb_w=spb, spb_w1=spb)
        cs.forward(x1, True)
        for k in range(3):
            g, gbf = (dh, 1) if k == 2 else (dx, 1)
            xin = cs.x1 if k == 0 else cs.z[k - 1]
            sp = None if k == 0 else cs.st[k - 1]

            def run():
                st = nat.stream_ptr(dev)   # the capture stream, not the one current outside it
                nat.check(cs._wgrad(k + 1, nat.ptr(xin), _ptr(sp), nat.ptr(g), gbf, nat.ptr(cs.z[k]),
                                    nat.ptr(cs.st[k]), nat.ptr(cs.wslab[k]), cs.N, cs.E, cs.B, cs.H, cs.W,
                                    cs.chunks_wl[k], cs.spb_wl[k], st), "wgrad")
            us = time_graph(run)
            print(json.dumps({"op": "wgrad", "layer": k + 1, "pilot": pilot, "spb": spb, "us": round(us, 1)}),
                  flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="qsc,conv")
    args = ap.parse_args()
    what = args.what.split(",")
    if "qsc" in what:
        grids = [(512, 256), (1024, 256), (1024, 512), (2304, 512), (2304, 768), (2304, 1152), (1024, 1024)]
        tune_qsc(8, 128, 2304, grids)
    if "wgrad" in what:
        tune_wgrad(128, 256, [4, 8, 16, 32])
    if "conv" in what:
        tune_conv(128, [256], list(itertools.product([1, 2, 4], [8], [4, 8])))


if __name__ == "__main__":
    main()
