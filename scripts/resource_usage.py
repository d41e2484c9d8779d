#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of a HIP source, from the compiler's
kernel-resource-usage remarks (CPU only: hipcc cross-compiles gfx950).

    python scripts/resource_usage.py csrc/hip/conv.hip [name-filter]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "quantum_distributed_machine_learning_ris_channel_estimation_amd")


def main():
    src = sys.argv[1]
    if not os.path.exists(src):
        src = os.path.join(PKG, src)
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    extra = sys.argv[3:] if len(sys.argv) > 3 else []
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast",
           "--offload-device-only", "-c", src, "-o", "/dev/null", "-I", os.path.join(PKG, "csrc", "hip"),
           "-Rpass-analysis=kernel-resource-usage"] + extra
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        txt = m.group(1).strip()
        if txt.startswith("Function Name:"):
            name = txt.split(":", 1)[1].strip()
            dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
            cur = {"name": dem}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    keys = ["VGPRs", "AGPRs", "VGPRs Spill", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
    print("| kernel | VGPR | AGPR | spill | waves/SIMD | static LDS |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        if flt in r["name"]:
            print(f"| `{r['name'][:110]}` | " + " | ".join(r.get(k, "?") for k in keys) + " |")


if __name__ == "__main__":
    main()
