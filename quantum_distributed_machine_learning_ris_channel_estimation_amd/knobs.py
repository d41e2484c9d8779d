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
    # (csrc/hip/gemm.hip; the rest on hipBLASLt), and their tile configurations (forward, wgrad, dgrad).
    # 8,7,6 (round 5) = the producer-wave tiles: isolated 33.0 / 38.8 / 35.1 us against 40.3 / 42.2 / 35.8 for round
    # 4's 6,1,2; in the step 0.3958-0.3967 against 0.3992-0.4025 ms (profiles/r5_02_gemm_probe.txt, r5_03_ab.txt)
    # "fwd" instead of "fwdplain": the forward with the loss in its epilogue (gemm.hip EPI_NMSE) where it tiles, else
    # the plain hand-written forward + the one-pass NMSE kernel.  Since the epilogue reduces its error sums per (batch,
    # expert) rather than per row the two are level: 0.3721 / 0.3726 against 0.3745 / 0.3737 ms on one box, 0.3842-
    # 0.3847 against 0.3839-0.3845 on another (profiles/r5_29_nmse_epilogue_ab.txt, r5_42_fused_fwd_ab.txt) -- the
    # plain forward stays.  (Shapes the epilogue does not tile fell back to hipBLASLt, whose forward breaks the
    # split-forward plans' equality with the serial step: profiles/r5_32_*, r5_41_map.txt, r5_42_library_fwd.log)
    hand_gemm: str = "fwdplain,wgrad,dgrad"
    gemm_cfg: str = "8,7,6"
    # fp8 estimator: the hand-written e4m3 forward (else torch._scaled_mm + the NMSE kernel), e4m3 FC gradients
    hand_fp8: bool = True
    f8_bwd: bool = True
    # the e4m3 GEMMs with producer waves (gemm.hip Geo PW = 4: loading waves beside the MFMA waves): forward 20.6 us
    # and data gradient 25.1 us isolated against 28.6 / 30.3; the fp8 step 0.3811-0.3819 ms against 0.3922-0.3946
    # (profiles/r5_05_*)
    f8_producers: bool = True
    # e4m3 convs for layers 2 / 3 of the fp8 estimator (opt-in: a net loss in the step, profiles/r2_14_*)
    fp8_conv: bool = False
    # the 8-qubit circuit forward on the matrix cores (csrc/hip/qsim_mfma.hip; else the register kernel)
    qsim_mfma: bool = True
    # layer 3's BN backward reduction in the FC data gradient's epilogue (gemm.hip BnRedEpi; else its own launch,
    # conv.hip bn_bwd_reduce_kernel)
    dgrad_bnred: bool = True
    # the same epilogue on the fp8 estimator's e4m3 data gradient (gemm.hip qd_gemm_dgrad_f8_bnred): 27.7 -> 36.9 us
    # alone against the 13 us launch it replaces; the fp8 step 0.3718-0.3730 against 0.3766-0.3772 ms
    # (profiles/r5_27_*; with the epilogue's rolled butterfly it was +17 us and no faster, r5_21 / r5_23)
    dgrad_bnred_f8: bool = True
    # the 12-qubit circuit, forward and adjoint, on the matrix cores (csrc/hip/qsim12_mfma.hip; else qsim_big.hip)
    qsim_mfma12: bool = True
    # the 8-qubit adjoint backward on the matrix cores (qsim12_mfma.hip qd_qsim_mfma8_bwd; else qsim.hip's)
    qsim_mfma_bwd: bool = True
    # (world 1) the HDCE Adam launch sums the step's gradient slabs (conv weights, BN, FC bias) in extra workgroups
    # (optim.hip AdamSlabs) instead of a slab-reduction launch before it on the chain.  Off: bit-identical but not
    # faster -- 0.3856-0.3876 against 0.3830-0.3852 ms with the slab workgroups first in block order, no gain with
    # them last (profiles/r5_19_adam_slabs_ab_v*.txt); the slab-fed variant needs 90 VGPRs (occupancy 5 for the
    # HBM-bound update instead of 7)
    adam_slabs: bool = False
    # the conv stack's training forward as one persistent launch (conv.hip conv_fwd_stack_kernel; else 3 conv launches
    # + the BN tail launch).  Measured slower: 105 against 58 us alone (docs/CONCURRENCY.md)
    conv_stack: bool = False
    # the QSC preprocess forward's workgroup cap (ops/qsc.py; one sample per wave beyond it, a grid-stride loop)
    qsc_fwd_cap: int = 256
    # P256: the QSC preprocess forward's conv2 on bf16x3 MFMAs too (qd_qsc2_fwd3).  Round 6's conv1 on MFMAs took
    # the P256 forward kernels to 186 / 193 VGPRs (2 waves per SIMD; before: 248 + 16, 1 wave), which the bf16x3
    # form was turned down for
    qsc_fwd3_p256: bool = False
    # conv stack launch shapes (ops/conv.py ConvStackHIP): samples per wave of the forward / dgrad kernels (4 waves per
    # workgroup), samples per workgroup of the fused layer-3/2 backward and of layer 1's weight gradient.
    # spw 3 (round 5): 198 workgroups, one per CU -- spw 2's 288 put two on 32 CUs, whose workgroups then set each
    # layer's time: 0.3869 / 0.3879 against 0.3909 / 0.3909 ms, and 0.4081 / 0.4066 against 0.4102 / 0.4084 on another
    # box (profiles/r5_18_spw_stack_window_ab.txt, r5_10_ab.txt)
    conv_spw: int = 3
    # (round 6) layers 2 / 3 of the P128 training forward on conv3x3_fwd_db_kernel: per wave, the next sample's staging
    # runs in the current sample's MFMA shadow (two LDS tiles); bit-identical to conv3x3_kernel
    conv_fwd_db: bool = False
    # (round 6) layers 3 / 2's fused backward at P128 on conv3x3_bwd_db_kernel (two stage buffers: the next sample staged
    # in the current one's MFMA shadow), conv_spb_db samples per workgroup -- 10: 234 workgroups, one per CU
    conv_bwd_db: bool = False
    conv_spb_db: int = 10
    # (round 6) the training / eval forward of all three layers on conv3x3_split_kernel: each sample split over a
    # workgroup's 4 waves (one position tile each), conv_sps (4..6) samples per workgroup, several workgroups per CU.
    # Off: level alone at P128 and 14 % faster at P256, but slower in both steps (P128 0.3834-0.3859 against
    # 0.3807-0.3827 ms, P256 1.105-1.109 against 1.089-1.092: profiles/r6_18_conv_split_ab.txt, r6_20_*)
    conv_fwd_split: bool = False
    conv_sps: int = 5
    # (round 6) layer 1 alone on conv3x3_split_kernel at 4 x conv_spw samples per workgroup (the statistics chunking of
    # conv3x3_kernel, so layers 2 / 3 and the BN tail are unchanged).  Off: level in the step, 0.3775-0.3820 against
    # 0.3768-0.3801 ms (profiles/r6_37_conv_l1_split_ab.txt)
    conv_l1_split: bool = False
    conv_spb_f: int = 5
    # (round 6) the same at P256 (W = 16): its fused backward holds 131 KB of LDS, one workgroup per CU, so spb 5's 468
    # workgroups ran in two rounds; 10 (234) is one -- the P256 step 1.109-1.118 against 1.128-1.138 ms alternating,
    # 1.077-1.078 against 1.098-1.103 on another box (profiles/r6_40_p256_conv_spb10_ab.txt, r6_38_*, r6_39_*)
    conv_spb_f_w16: int = 10
    conv_spb_w1: int = 4


KNOBS = Knobs()
