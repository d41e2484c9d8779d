"""What does ds_read_b64_tr_b8 deliver?  LDS byte a holds a & 0xff; a 16-lane group reads an 8-row x 16-column
byte block of pitch 16 (value = 16 row + col).  Hypothesis: lane 2q + p supplies row q, columns 8p .. 8p + 7,
and lane i receives column i of the 8 rows (byte q = row q)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import ctypes  # noqa: E402

import torch  # noqa: E402

from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    fill = (torch.arange(4096, dtype=torch.int32) % 256).to(torch.uint8).to(dev)
    addr = torch.tensor([(l % 16) // 2 * 16 + 8 * (l % 2) for l in range(64)], dtype=torch.int32, device=dev)
    out = torch.zeros(512, dtype=torch.uint8, device=dev)
    f = nat.fn(nat.hip_lib(), "qd_tr_b8_probe", [ctypes.c_void_p] * 4)
    nat.check(f(nat.ptr(addr), nat.ptr(out), nat.ptr(fill), nat.stream_ptr(dev)), "tr_b8_probe")
    o = out.view(64, 8).cpu().tolist()
    for l in range(16):
        print(l, o[l])
    ok = all(o[l][j] == 16 * j + (l % 16) for l in range(64) for j in range(8))
    print("hypothesis (lane i <- column i, byte q <- row q):", ok)


if __name__ == "__main__":
    main()
