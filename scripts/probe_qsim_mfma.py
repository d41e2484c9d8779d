"""Isolated timing: 8-qubit forward on the matrix cores (qsim_mfma.hip) vs the register kernel
(qsim.hip), flagship shape (9 QuantumNAT groups x 256 samples, 3 layers), with and without the saved
final state.   python scripts/probe_qsim_mfma.py"""
import ctypes
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat  # noqa: E402

cuda = torch.device("cuda", 0)
lib = nat.hip_lib()
_p, _i = ctypes.c_void_p, ctypes.c_int
G, b, L = 9, 256, 3
B = G * b
x = torch.rand(B, 8, device=cuda) * 2 - 1
w = torch.rand(G, L, 8, 2, device=cuda) * 6.28
E = torch.empty(B, 8, device=cuda)
ps = torch.empty(B * 512, device=cuda)
ops = torch.empty(nat.fn(lib, "qd_qsim_mfma_ops_halves", [_i, _i], ctypes.c_longlong)(G, L), dtype=torch.float16,
                  device=cuda)
st = nat.stream_ptr(cuda)
reg = nat.fn(lib, "qd_qsim_fwd_save", [_p, _p, _p, _i, _i, _i, _i, _p, _p])
prep = nat.fn(lib, "qd_qsim_mfma_prep", [_p, _p, _i, _i, _p])
mf = nat.fn(lib, "qd_qsim_mfma_fwd", [_p, _p, _p, _p, _i, _i, _i, _p, _p])
cases = {
    "register": lambda: reg(nat.ptr(x), nat.ptr(w), nat.ptr(E), B, 8, L, b, nat.ptr(ps), st),
    "mfma(prep+fwd)": lambda: (prep(nat.ptr(w), nat.ptr(ops), G, L, st),
                               mf(nat.ptr(x), nat.ptr(w), nat.ptr(ops), nat.ptr(E), B, L, b, nat.ptr(ps), st)),
    "mfma(fwd only)": lambda: mf(nat.ptr(x), nat.ptr(w), nat.ptr(ops), nat.ptr(E), B, L, b, nat.ptr(ps), st),
}
for name, f in cases.items():
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(200):
        ev[0].record()
        f()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
    ts.sort()
    print(f"{name:16s} median {ts[len(ts) // 2]:7.2f} us  min {ts[0]:7.2f} us", flush=True)
