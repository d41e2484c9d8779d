#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy summary of one .hip file (hipcc -Rpass-analysis)."""
import re, subprocess, sys
src = sys.argv[1]
extra = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
       "-I", "/root/repo/quantum_distributed_machine_learning_ris_channel_estimation_amd/csrc/hip", "-c", src,
       "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
cur = {}
for ln in out.splitlines():
    m = re.search(r"remark: (.*)", ln)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        if cur:
            print(cur)
        name = t.split(":", 1)[1].strip()
        g = re.search(r"Geo<([^>]*)>, (\d+), (\d+), (\d+)", name)
        cur = {"k": g.group(0) if g else name[:90]}
    else:
        for key in ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"):
            if t.startswith(key + ":"):
                cur[key.split()[0]] = t.split(":", 1)[1].strip()
if cur:
    print(cur)
