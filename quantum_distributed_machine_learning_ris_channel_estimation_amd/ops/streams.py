"""CU-masked HIP streams: give a concurrent branch of the training step a fixed share of the chip.

``masked_stream(cus)`` wraps ``hipExtStreamCreateWithCUMask`` (csrc/hip/runtime.hip) as a
``torch.cuda.ExternalStream``; ``cu_probe`` launches a kernel that records the hardware id of every
workgroup, so the mask's effect (and whether a HIP graph replay keeps it) is measured, not assumed.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable, List, Tuple

import torch

from .. import _native as nat

_p, _i = ctypes.c_void_p, ctypes.c_int
_live: Dict[int, "torch.cuda.ExternalStream"] = {}   # masked streams live for the process


def mask_words(cus: Iterable[int], n_cu: int) -> List[int]:
    words = [0] * ((n_cu + 31) // 32)
    for c in cus:
        if not 0 <= c < n_cu:
            raise ValueError(f"CU {c} outside 0..{n_cu - 1}")
        words[c // 32] |= 1 << (c % 32)
    return words


def parse_cus(spec: str, n_cu: int) -> List[int]:
    """``spec``: ``a-b`` (range), ``a,b,c`` (list), ``stride:S:O[:N]`` (every S-th CU from O, N of them),
    ``first:N``; ``+``-joined specs are unioned."""
    out = set()
    for part in spec.split("+"):
        part = part.strip()
        if part.startswith("first:"):
            out.update(range(int(part[6:])))
        elif part.startswith("stride:"):
            f = [int(v) for v in part[7:].split(":")]
            s, o = f[0], f[1]
            n = f[2] if len(f) > 2 else (n_cu - o + s - 1) // s
            out.update(o + s * i for i in range(n))
        else:
            for tok in part.split(","):
                if "-" in tok:
                    a, b = tok.split("-")
                    out.update(range(int(a), int(b) + 1))
                elif tok:
                    out.add(int(tok))
    return sorted(out)


def masked_stream(cus: Iterable[int], device=None) -> "torch.cuda.ExternalStream":
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = mask_words(cus, n_cu)
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = ctypes.c_void_p()
    with torch.cuda.device(dev):
        f = nat.fn(nat.hip_lib(), "qd_stream_create_cu_mask", [_p, _i, ctypes.POINTER(ctypes.c_void_p)])
        nat.check(f(arr, len(words), ctypes.byref(h)), "hipExtStreamCreateWithCUMask")
    s = torch.cuda.ExternalStream(h.value, device=dev)
    _live[h.value] = s
    return s


def stream_mask(stream, n_cu: int) -> List[int]:
    nw = (n_cu + 31) // 32
    arr = (ctypes.c_uint32 * nw)()
    f = nat.fn(nat.hip_lib(), "qd_stream_get_cu_mask", [_p, ctypes.POINTER(ctypes.c_uint32), _i])
    nat.check(f(ctypes.c_void_p(stream.cuda_stream), arr, nw), "hipExtStreamGetCUMask")
    return [c for c in range(n_cu) if arr[c // 32] >> (c % 32) & 1]


def cu_probe_launch(out: torch.Tensor, spin: int = 64) -> None:
    """Launch the probe on the current stream: one 64-thread workgroup per (hw_id, xcc_id) pair of ``out``."""
    assert out.dtype == torch.int32 and out.is_cuda and out.numel() % 2 == 0
    f = nat.fn(nat.hip_lib(), "qd_cu_probe", [_p, _i, _i, _p])
    nat.check(f(nat.ptr(out), out.numel() // 2, spin, nat.stream_ptr(out.device)), "qd_cu_probe")


def decode(out: torch.Tensor) -> List[Tuple[int, int, int, int]]:
    """(xcc, shader engine, shader array, cu) of every probe record (gfx9 HW_ID layout)."""
    v = out.view(-1, 2).cpu().tolist()
    res = []
    for hw, xcc in v:
        hw &= 0xFFFFFFFF
        res.append((xcc & 0xF, (hw >> 13) & 0x7, (hw >> 12) & 1, (hw >> 8) & 0xF))
    return res
