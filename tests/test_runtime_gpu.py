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
