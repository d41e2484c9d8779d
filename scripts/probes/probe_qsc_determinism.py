"""Is the QSC step itself deterministic when other work shares the chip?  (docs/CONCURRENCY.md: the QSC-only
run-to-run mismatch.)  No cross-queue data at all: fixed inputs, the QuantumNAT counter reset before every run,
the whole QSC step (noise, preprocess CNN, 8-qubit simulator forward / adjoint, head, slabs) on one stream, and a
perturbing kernel on a second stream that changes size every run.  Every run's gradient, loss and simulator
state must equal the first run's bit for bit; a difference means a race inside a QSC kernel (timing-dependent),
not a stale read across queues.

    probe_qsc_determinism.py [runs]
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import QSC_P128  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.optim import FlatParamSpace  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.slabsum import SlabBatch  # noqa: E402
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import ClassifierStep  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda")
    torch.manual_seed(0)
    S, B = 9, 256
    qsc = QSC_P128(8, 3, 3, True, False, 128).to(dev)
    space = FlatParamSpace(list(qsc.named_parameters()), dev)
    skip = torch.zeros(64, device=dev)
    cs = ClassifierStep(qsc, S, space=space, batch_total=S * B, skip=skip[0:1], hip_kw={"grid_bwd": 256})
    cs.skip_add = False
    cs.writes_grads = cs.hip is not None
    assert cs.hip is not None, "HIP QSC step required"
    x = torch.randn(S * B, 2, 16, 8, device=dev)
    labels = torch.randint(0, 3, (S * B,), device=dev)
    ctr0 = cs.hip.noise_ctr.clone()
    busy = nat.fn(nat.hip_lib(), "qd_coh_busy", [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_void_p])
    junk = torch.rand(1 << 24, device=dev)
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    side = torch.cuda.Stream()
    slabs = SlabBatch()

    def one(r):
        cs.hip.noise_ctr.copy_(ctr0)
        space.grad.zero_()
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):   # perturbation: a different mix every run (GEMMs take whole CUs' LDS)
            for k in range(1 + r % 4):
                if (r + k) % 2:
                    torch.mm(a, a)
                else:
                    nat.check(busy(nat.ptr(junk), junk.numel() >> (r % 3), 8 + 8 * (r % 5), 256 << (r % 3),
                                   nat.stream_ptr()), "busy")
        q = cs(x, labels, slabs=slabs)
        slabs.launch(accumulate=False, stream=nat.stream_ptr(dev))
        main.wait_stream(side)
        torch.cuda.synchronize()
        return [space.grad.clone(), q.detach().reshape(-1).clone()] + \
            [t.clone() for t in (getattr(cs.hip, "psave", None), getattr(cs.hip, "E", None)) if t is not None]

    ref = one(0)
    bad = 0
    for r in range(1, runs):
        out = one(r)
        diff = [i for i, (u, v) in enumerate(zip(ref, out)) if not torch.equal(u, v)]
        if diff:
            bad += 1
            g = (ref[0] - out[0]).abs().max().item()
            print(f"run {r}: differs in outputs {diff} (max |dgrad| {g:.3e})", flush=True)
    print(f"{bad} / {runs - 1} runs differ from run 0 (outputs compared: grad, loss"
          f"{', psave' if getattr(cs.hip, 'psave', None) is not None else ''}"
          f"{', E' if getattr(cs.hip, 'E', None) is not None else ''})", flush=True)


if __name__ == "__main__":
    main()
