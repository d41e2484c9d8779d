"""The device clock stamps the one-graph DP plan's phase timing is built from (csrc/hip/runtime.hip
qd_stamp / qd_wallclock_khz; train/flagship_dp.py DPPlan._stamped_rows): stamps are stream-ordered, the
clock rate is known, and the interval between two stamps agrees with HIP events around the same work --
eagerly and replayed from a captured graph."""
import ctypes

import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat

pytestmark = pytest.mark.gpu


def _stamp(buf, i):
    f = nat.fn(nat.hip_lib(), "qd_stamp", [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p])
    nat.check(f(nat.ptr(buf), i, nat.stream_ptr()), "qd_stamp")


def _khz(cuda):
    k = ctypes.c_int(0)
    f = nat.fn(nat.hip_lib(), "qd_wallclock_khz", [ctypes.c_int, ctypes.POINTER(ctypes.c_int)])
    nat.check(f(cuda.index or 0, ctypes.byref(k)), "qd_wallclock_khz")
    return k.value


def test_clock_stamps_time_stream_ordered_work(cuda):
    khz = _khz(cuda)
    assert 1_000 <= khz <= 10_000_000   # (MHz-class constant clock)
    a = torch.randn(4096, 4096, device=cuda, dtype=torch.bfloat16)
    buf = torch.zeros(4, dtype=torch.int64, device=cuda)

    def work():
        _stamp(buf, 0)
        for _ in range(8):
            torch.mm(a, a)
        _stamp(buf, 1)

    work()   # (warm: library load, first-launch costs)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    work()
    e1.record()
    torch.cuda.synchronize()
    t = buf.tolist()
    stamp_ms, ev_ms = (t[1] - t[0]) / khz, e0.elapsed_time(e1)
    assert t[1] > t[0] > 0
    assert 0.5 * ev_ms <= stamp_ms <= 1.05 * ev_ms + 0.05, (stamp_ms, ev_ms)

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        work()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        work()
    buf.zero_()
    g.replay()
    torch.cuda.synchronize()
    t2 = buf.tolist()
    assert t2[1] > t2[0] > t[1]
    assert (t2[1] - t2[0]) / khz >= 0.5 * ev_ms


def test_packed_f32_war_probe_plain_fma_is_safe(cuda):
    """csrc/hip/hazard_probe.hip (round 6): the instruction pattern of the QSC preprocess forward's misread -- an
    FMA reading registers that the next ds_read rewrites -- with MFMA partner waves on every SIMD.  With plain
    v_fma_f32 (what the library is built to emit: _native.NO_PACKED_F32) the result is wave-uniform in every
    iteration.  (The packed form is only reported, not asserted: profiles/r6_03_pkfma_war.txt.)"""
    import ctypes
    import torch
    from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
    f = nat.fn(nat.hip_lib(), "qd_pkfma_war_probe", [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p])
    res = {}
    for mode in (2 | 1, 1):
        out = torch.zeros(132, dtype=torch.int32, device=cuda)
        nat.check(f(mode, 500, 256, nat.ptr(out), nat.stream_ptr(out.device)), "pkfma_war_probe")
        torch.cuda.synchronize()
        res[mode] = (int(out[0]), int(out[1]))
    print("pkfma WAR probe (events, iterations):", res)
    assert res[3][1] == 500 * 256 * 4 and res[3][0] == 0
