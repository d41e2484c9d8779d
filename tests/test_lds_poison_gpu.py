"""Uninitialised-LDS sanitizer (SURVEY §5.2 race detection): every hand-written kernel of a training step
must read only LDS it wrote in its own launch.

LDS is not cleared between workgroups.  A kernel that reads a pad row or a tail it never wrote sees
whatever the CU's previous workgroup left there: usually its own predecessor's data (so the bug is
invisible in a serial run), but another kernel's data when two streams interleave on the CUs -- a
run-to-run difference that appears only under concurrency.  In poison mode (``_native.set_lds_poison``)
every launch is preceded on its stream by a grid that fills the whole LDS of every CU with a pattern;
the poisoned run must then be bit-identical to a clean one.  Two patterns: all-ones (NaN in fp32, bf16
and e4m3: caught by any arithmetic use) and 0x7F7F7F7F (a huge finite fp32 / bf16 value: caught by
max-pool / ReLU reads, which drop NaNs)."""
import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
from quantum_distributed_machine_learning_ris_channel_estimation_amd.parallel.dp import DistContext
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.flagship import FlagshipConfig, FlagshipTrainer

pytestmark = pytest.mark.gpu


def _state(tr):
    return [tr.hdce.space.flat, tr.qspace.flat, tr.hopt.m, tr.hopt.v, tr.qopt.m, tr.qopt.v, tr.hloss, tr.qloss] + \
        list(tr.hdce.run_mean) + list(tr.hdce.run_var)


def _train(cuda, kw, steps, pattern=None):
    nat.set_lds_poison(pattern)
    try:
        cfg = FlagshipConfig(hip_graphs=False, stream_mode="serial", qsc_grid_bwd=128, **kw)
        tr = FlagshipTrainer(cfg, DistContext(device=cuda))
        for _ in range(steps):
            tr.step()
        torch.cuda.synchronize()
        return [t.detach().clone() for t in _state(tr)]
    finally:
        nat.set_lds_poison(None)


CONFIGS = {
    "p128_q8_bf16": dict(batch=32, data_len=800),
    "p128_q8_fp8": dict(batch=32, data_len=800, dtype="fp8"),
    "p256_q12": dict(batch=16, data_len=400, pilot_num=256, n_qubits=12),
    "p128_q16": dict(batch=4, data_len=200, n_qubits=16),
}


@pytest.mark.parametrize("name", list(CONFIGS))
def test_poisoned_lds_changes_nothing(cuda, name):
    kw = CONFIGS[name]
    ref = _train(cuda, kw, 3)
    for pattern in (0xFFFFFFFF, 0x7F7F7F7F):
        got = _train(cuda, kw, 3, pattern)
        for i, (a, b) in enumerate(zip(ref, got)):
            assert torch.equal(a, b), (name, hex(pattern), i, float((a.float() - b.float()).abs().max()))


def test_poison_reaches_every_launch(cuda):
    """The hook really runs: a kernel that reads LDS it never wrote (qd_lds_peek) returns the pattern."""
    import ctypes
    for pattern in (0x3F800000, 0xFFFFFFFF):
        nat.set_lds_poison(pattern)
        try:
            out = torch.zeros(64, dtype=torch.int64, device=cuda)
            o32 = torch.zeros(64, dtype=torch.int32, device=cuda)
            f = nat.fn(nat.hip_lib(), "qd_lds_peek", [ctypes.c_void_p, ctypes.c_void_p])
            nat.check(f(nat.ptr(o32), nat.stream_ptr(cuda)), "lds_peek")
            torch.cuda.synchronize()
            out = o32.to(torch.int64) & 0xFFFFFFFF
            assert bool((out == pattern).all()), [hex(int(v)) for v in out[:4]]
        finally:
            nat.set_lds_poison(None)
