"""Round 6: no packed-FP32 VALU instruction anywhere in the kernel library except the hazard probe.

On gfx950 a v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 whose source registers are rewritten by a younger LDS read
can read the new value in its last quarter-wave (lanes 48-63) while another wave on its SIMD issues MFMAs
(csrc/hip/hazard_probe.hip; profiles/r6_03_pkfma_war.txt: 44,687 of 2,048,000 iterations with MFMA partners, 0
without, 0 with plain v_fma_f32).  That was the QSC preprocess forward's lanes-48..63 misread (docs/CONCURRENCY.md),
and the compiler forms these instructions on its own -- so the library is built without them (_native.py
NO_PACKED_F32).  This test disassembles every gfx950 code object inside libqdml_hip.so (CPU only)."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "quantum_distributed_machine_learning_ris_channel_estimation_amd", "lib", "libqdml_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
PACKED = re.compile(r"\bv_pk_(fma|mul|add)_f32\b")


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump missing")
def test_only_the_hazard_probe_has_packed_f32(tmp_path):
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, capture_output=True, cwd=tmp_path)
    objs = [p for p in os.listdir(tmp_path) if "amdgcn" in p and "gfx950" in p]
    assert objs, os.listdir(tmp_path)
    hits, fns = {}, 0
    for o in objs:
        dis = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", str(tmp_path / o)], check=True,
                             capture_output=True, text=True).stdout
        fn = None
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                fn, fns = m.group(1), fns + 1
            elif fn and PACKED.search(line):
                hits[fn] = hits.get(fn, 0) + 1
    assert fns > 100   # (the whole library was read)
    assert hits, "the hazard probe's packed FMAs should be there (it is built with them on purpose)"
    assert all("pkfma_war_probe" in f for f in hits), {f: n for f, n in hits.items() if "pkfma_war_probe" not in f}
