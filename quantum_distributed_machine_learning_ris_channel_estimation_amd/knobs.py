"""Kernel-path switches of the HIP engine that tests flip (Python attributes, not environment variables).

Every default is the measured-fastest choice on MI355X; the alternatives stay because a test pins one path
against the other (hand-written vs library GEMM, e4m3 vs bf16 gradients, ...).  Alternatives that were
measured slower and that no test needs were removed in round 4 -- their measurements are in docs/ and
profiles/.  Tests change a switch with ``monkeypatch.setattr(knobs.KNOBS, name, value)`` before building the
engine that reads it.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class Knobs:
    # FC GEMMs (train/engine.py HDCEStep): which of forward / wgrad / dgrad run on the hand-written kernels
    # (csrc/hip/gemm.hip; the rest on hipBLASLt), and their tile configurations (forward, wgrad, dgrad)
    hand_gemm: str = "fwdplain,wgrad,dgrad"
    gemm_cfg: str = "6,1,2"
    # fp8 estimator: the hand-written e4m3 forward (else torch._scaled_mm + the NMSE kernel), e4m3 FC gradients
    hand_fp8: bool = True
    f8_bwd: bool = True
    # e4m3 convs for layers 2 / 3 of the fp8 estimator (opt-in: a net loss in the step, profiles/r2_14_*)
    fp8_conv: bool = False
    # the 8-qubit circuit forward on the matrix cores (csrc/hip/qsim_mfma.hip; else the register kernel)
    qsim_mfma: bool = True


KNOBS = Knobs()
