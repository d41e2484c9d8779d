"""Build and load the framework's native code.

Two shared objects are produced IN-TREE under ``<pkg>/lib`` (so they travel with a
repo snapshot to a GPU box):

* ``libqdml_hip.so`` -- every ``csrc/hip/*.hip`` kernel, compiled by ``hipcc
  --offload-arch=gfx950`` (CDNA4 only; no CUDA / hipify / dual paths).  Launchers
  are ``extern "C"`` functions taking raw device pointers and a ``hipStream_t``;
  they enqueue on torch's current stream, so they are captured by HIP graphs
  like any other kernel.
* ``libqdml_cpu.so`` -- the C++/OpenMP runtime pieces (CPU state-vector simulator,
  host data utilities).

The HIP library links ``libamdhip64.so.7``; torch must be imported first so the
dynamic loader binds that SONAME to the HIP runtime torch already loaded (one
runtime per process, shared streams).
"""
from __future__ import annotations

import ctypes
import os
import shutil
import subprocess
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_DIR = os.environ.get("QDML_LIB_DIR") or os.path.join(PKG_DIR, "lib")   # (override: A/B builds side by side)
OBJ_DIR = os.path.join(LIB_DIR, "obj")
HIP_LIB = os.path.join(LIB_DIR, "libqdml_hip.so")
CPU_LIB = os.path.join(LIB_DIR, "libqdml_cpu.so")
ARCH = os.environ.get("QDML_OFFLOAD_ARCH", "gfx950")

_lock = threading.Lock()
_hip: Optional[ctypes.CDLL] = None
_cpu: Optional[ctypes.CDLL] = None


class NativeUnavailable(RuntimeError):
    pass


def _sources(sub: str, ext: str) -> List[str]:
    d = os.path.join(CSRC, sub)
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(ext))


def _headers(sub: str) -> List[str]:
    d = os.path.join(CSRC, sub)
    return [os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp", ".cuh"))]


def _stale(target: str, deps: List[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print("[qdml build]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")


def hipcc() -> Optional[str]:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    return None


# gemm.hip: MFMA accumulators in VGPRs (the default AGPR form made hipcc shuttle the 18-36 accumulator
# tiles between the register files every K step)
# qsim_stream.hip: no SLP vectorisation (packed-f32 pairs of the complex gate math doubled the register
# demand: the adjoint passes spilled at 256 VGPRs, 86-92 without)
# hazard_probe.hip: the one file WITH packed-FP32 instructions (its inline asm demonstrates their hazard; see below)
# qsim_stream.hip also without the SI load/store optimizer: it pairs the streamed passes' 8-byte LDS accesses into
# ds_read2_b64 / ds_write2_b64, whose banks wrap every 32 dwords -- 24 % of the reverse pass A's LDS cycles were bank
# conflicts (profiles/r6_54_qstream_pmc_b.md); single ds_read_b64 bank on 64 (QDML_QSTREAM_LSO=1: the paired build)
_QS_LSO = [] if os.environ.get("QDML_QSTREAM_LSO") == "1" else ["-Xclang", "-target-feature", "-Xclang", "-load-store-opt"]
PER_FILE_FLAGS = {"gemm.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"], "qsim_stream.hip": ["-fno-slp-vectorize"] + _QS_LSO,
                  "qsim_mfma.hip": ["-fno-slp-vectorize"], "qsim12_mfma.hip": ["-fno-slp-vectorize"],
                  "hazard_probe.hip": ["-Xclang", "-target-feature", "-Xclang", "+packed-fp32-ops"]}
# (measurement) more files without the SI load/store optimizer: QDML_NOLSO_FILES="a.hip,b.hip"
for _f in filter(None, os.environ.get("QDML_NOLSO_FILES", "").split(",")):
    PER_FILE_FLAGS[_f] = PER_FILE_FLAGS.get(_f, []) + ["-Xclang", "-target-feature", "-Xclang", "-load-store-opt"]
# No packed-FP32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) anywhere else (round 6).  On gfx950 a packed-FP32
# instruction whose source registers are rewritten by a younger LDS read can -- while another wave on its SIMD is
# issuing MFMAs -- read the NEW value in its last quarter-wave (lanes 48-63): 44,687 of 2,048,000 probe iterations
# with MFMA partners, 0 without, 0 with plain v_fma_f32 (csrc/hip/hazard_probe.hip, profiles/r6_03_pkfma_war.txt).
# That was the QSC preprocess forward's lanes-48..63 misread (docs/CONCURRENCY.md).  The compiler forms these
# instructions on its own (vector types, SLP), so the feature is off for the whole library.
NO_PACKED_F32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
if os.environ.get("QDML_PACKED_F32") == "1":   # (measurement only: the hazard-exposed build, for its A/B)
    NO_PACKED_F32 = []


def build_hip(force: bool = False, verbose: bool = True, jobs: int = 8) -> str:
    cc = hipcc()
    if cc is None:
        raise NativeUnavailable("hipcc not found")
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = _sources("hip", ".hip")
    hdrs = _headers("hip")
    flags = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
             "-Wno-unused-result", "-I", os.path.join(CSRC, "hip")] + NO_PACKED_F32
    flags += os.environ.get("QDML_HIPCC_EXTRA", "").split()   # (tuning sweeps: extra -D defines)
    # a changed flag set (a tuning build, then the default again) rebuilds every object
    stamp = os.path.join(OBJ_DIR, "flags.txt")
    want = " ".join(f for f in flags if not f.startswith("/"))   # (not the include path: the tree moves)
    want += " " + repr(sorted(PER_FILE_FLAGS.items()))
    if not force and (not os.path.exists(stamp) or open(stamp).read() != want):
        force = True
    objs = []

    def one(src: str) -> str:
        obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
        if force or _stale(obj, [src] + hdrs):
            _run([cc] + flags + PER_FILE_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj], verbose)
        return obj

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(one, srcs))
    if force or _stale(HIP_LIB, objs):
        _run([cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", HIP_LIB] + objs, verbose)
    with open(stamp, "w") as f:
        f.write(want)
    return HIP_LIB


def build_cpu(force: bool = False, verbose: bool = True) -> str:
    cxx = os.environ.get("CXX", shutil.which("g++") or "g++")
    srcs = _sources("cpu", ".cpp")
    os.makedirs(LIB_DIR, exist_ok=True)
    if force or _stale(CPU_LIB, srcs + _headers("cpu")):
        _run([cxx, "-O3", "-std=c++17", "-fopenmp", "-fPIC", "-shared", "-o", CPU_LIB] + srcs, verbose)
    return CPU_LIB


def build_all(force: bool = False, verbose: bool = True) -> None:
    build_cpu(force, verbose)
    build_hip(force, verbose)


def _declare(lib: ctypes.CDLL) -> None:
    # All launchers return an int status (hipError_t) and take pointers / ints /
    # floats; declare argtypes lazily in ops modules via `fn()`.
    pass


def hip_lib(build_if_missing: bool = True) -> ctypes.CDLL:
    """The HIP kernel library.  Raises if it cannot be loaded (no silent fallback)."""
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is not None:
            return _hip
        import torch  # noqa: F401  (bind libamdhip64.so.7 to torch's runtime first)
        if not os.path.exists(HIP_LIB):
            if not build_if_missing:
                raise NativeUnavailable(f"{HIP_LIB} missing; run __graft_entry__.build()")
            build_hip(verbose=False)
        lib = ctypes.CDLL(HIP_LIB, mode=ctypes.RTLD_GLOBAL)
        # native frames on a host crash (csrc/hip/runtime.hip qd_install_crash_handler), ahead of faulthandler
        if os.environ.get("QDML_CRASH_HANDLER", "1") == "1" and hasattr(lib, "qd_install_crash_handler"):
            lib.qd_install_crash_handler()
        _hip = lib
    return _hip


def cpu_lib(build_if_missing: bool = True) -> ctypes.CDLL:
    global _cpu
    if _cpu is not None:
        return _cpu
    with _lock:
        if _cpu is not None:
            return _cpu
        if not os.path.exists(CPU_LIB):
            if not build_if_missing:
                raise NativeUnavailable(f"{CPU_LIB} missing")
            build_cpu(verbose=False)
        _cpu = ctypes.CDLL(CPU_LIB)
    return _cpu


def check(status: int, what: str) -> None:
    if status != 0:
        raise RuntimeError(f"{what} failed with HIP status {status}")


def fn(lib: ctypes.CDLL, name: str, argtypes, restype=ctypes.c_int):
    f = getattr(lib, name)
    if getattr(f, "_qd_declared", False) is False:
        f.argtypes = argtypes
        f.restype = restype
        f._qd_declared = True
    if _POISON is None or name.startswith("qd_lds_poison"):
        return f
    return _poisoned(f)


# ---------------------------------------------------------------- LDS poisoning (sanitizer)
# Uninitialised-LDS detector.  LDS is not cleared between workgroups, so a kernel that reads LDS it
# did not write this launch sees whatever the CU's previous workgroup left there -- usually the same
# kernel's data (a pad row zeroed by its predecessor), but a different kernel's when two streams
# interleave on the CUs: a run-to-run difference that appears only under concurrency.  In poison mode
# every launch made through fn() on a stream handed out by stream_ptr() is preceded, on that stream, by
# a grid that fills the whole LDS of every CU with a pattern (csrc/hip/runtime.hip lds_poison_kernel);
# results must be bit-identical to an unpoisoned run (tests/test_lds_poison_gpu.py).
_POISON = None            # None, or the 32-bit fill pattern
_POISON_STREAMS = set()   # stream handles stream_ptr() returned while poisoning


def set_lds_poison(pattern) -> None:
    """Enable (a 32-bit pattern, e.g. 0xFFFFFFFF = NaN in fp32 / bf16 / e4m3) or disable (None) LDS
    poisoning for the launchers declared from now on (ops objects cache their launchers at construction:
    build them after this call)."""
    global _POISON
    _POISON = None if pattern is None else int(pattern) & 0xFFFFFFFF
    _POISON_STREAMS.clear()


def _poisoned(f):
    def call(*args):
        st = args[-1] if args else None
        if _POISON is not None and isinstance(st, ctypes.c_void_p) and st.value in _POISON_STREAMS:
            lp = fn(hip_lib(), "qd_lds_poison", [ctypes.c_uint32, ctypes.c_void_p])
            check(lp(_POISON, st), "qd_lds_poison")
        return f(*args)
    return call


def stream_ptr(device=None) -> ctypes.c_void_p:
    import torch
    h = torch.cuda.current_stream(device).cuda_stream
    v = ctypes.c_void_p(h)
    if _POISON is not None:
        _POISON_STREAMS.add(v.value)   # (the null stream's handle is 0: c_void_p(0).value is None)
    return v


def ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())
