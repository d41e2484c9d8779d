"""LS and LMMSE channel-estimation baselines.

Reference: ``generate_data.generate_MMSE_estimate(HLS, sigma2)`` (called at Test.py:145,
not shipped).  It refines the full-grid LS estimate given the pilot noise variance
``sigma2 = 10^(-snr/10)``.  We implement linear MMSE with a channel covariance learned
from the synthetic generator:

  H_mmse = W HLS,  W = R (R + s2_LS I)^-1,  s2_LS = sigma2 * 10^(LS_GAIN_DB/10)

``mode='freq'`` (default) uses the 16x16 subcarrier covariance per RIS element (the
classic OFDM LMMSE); ``mode='full'`` the full 1024x1024 covariance.  The filter is
applied as a complex GEMM (on the GPU when the input is there).

``mode='subspace'`` is the reference-calibrated baseline: the reference's MMSE curve (FIG1) sits a
constant ~1.4 dB below LS at every SNR, the signature of a fixed-rank projection rather
than a Wiener filter (whose gain vanishes at high SNR).  It projects each RIS element's 16-subcarrier LS
vector onto the top-``rank`` eigenvectors of the subcarrier covariance (the DFT-truncation estimator
with a learned basis): noise power x rank/16, rank 12 -> LS - 1.25 dB when the channel lies in that
subspace.  ``evaluate`` reports it as the FIG1 "MMSE" row and the LMMSE alongside.
"""
from __future__ import annotations

from functools import lru_cache
from typing import Optional

import numpy as np
import torch

from .channel import H_DIM, LS_GAIN_DB, N_ELEM, N_SUBC, generate_mixed


def covariance(H: torch.Tensor, mode: str = "freq") -> torch.Tensor:
    if mode == "freq":
        h = H.reshape(-1, N_ELEM, N_SUBC).reshape(-1, N_SUBC)
        return (h.T @ h.conj()) / h.shape[0]          # R[f, f'] = E[h_f h_f'^*]
    if mode == "full":
        return (H.T @ H.conj()) / H.shape[0]
    raise ValueError(mode)


SUBSPACE_RANK = 12


def subspace_matrix(R: torch.Tensor, rank: int = SUBSPACE_RANK) -> torch.Tensor:
    """P = U_r U_r^H, U_r the top-``rank`` eigenvectors of R."""
    R = R.to(torch.complex128)
    evals, U = torch.linalg.eigh(R)        # ascending
    Ur = U[:, -rank:]
    return Ur @ Ur.conj().T


def lmmse_matrix(R: torch.Tensor, noise_var: float) -> torch.Tensor:
    """W = R (R + s2 I)^-1 computed via the Hermitian eigendecomposition."""
    R = R.to(torch.complex128)
    evals, U = torch.linalg.eigh(R)
    evals = evals.clamp_min(0)
    gain = evals / (evals + noise_var)
    return (U * gain.to(U.dtype)) @ U.conj().T


def apply_lmmse(HLS: torch.Tensor, W: torch.Tensor, mode: str = "freq") -> torch.Tensor:
    W = W.to(device=HLS.device, dtype=torch.complex64)
    if mode == "freq":
        h = HLS.reshape(-1, N_ELEM, N_SUBC)
        return (h @ W.T).reshape(-1, H_DIM)
    return HLS @ W.T


@lru_cache(maxsize=4)
def _calibration_covariance(mode: str, n: int = 4096, seed: int = 7) -> torch.Tensor:
    _, _, H, _ = generate_mixed(n, snr_db=100.0, index=-1, base_seed=seed, split="calib")
    return covariance(H, mode)


def lmmse_estimate(HLS: torch.Tensor, sigma2: float, mode: str = "freq",
                   R: Optional[torch.Tensor] = None) -> torch.Tensor:
    if mode == "subspace":
        R = _calibration_covariance("freq") if R is None else R
        return apply_lmmse(HLS, subspace_matrix(R), "freq")
    R = _calibration_covariance(mode) if R is None else R
    W = lmmse_matrix(R, sigma2 * 10 ** (LS_GAIN_DB / 10))
    return apply_lmmse(HLS, W, mode)


def generate_MMSE_estimate(HLS_np, sigma2: float, mode: str = "freq"):
    """Reference-compatible signature (Test.py:145): complex ndarray in, complex ndarray out."""
    HLS = torch.as_tensor(np.asarray(HLS_np)).to(torch.complex64)
    return lmmse_estimate(HLS, sigma2, mode).numpy()
