"""Synthetic DeepMIMO-shaped RIS/OFDM channel generator.

The reference imports ``generate_data`` (Runner_P128_QuantumNAT_onchipQNN.py:16,
Test.py:7) but does not ship it, nor the DeepMIMO-derived ``available_data/*.npy``
(R:48-55).  This module supplies a generator with the same *interfaces and shapes*:

* a channel ``H`` has 1024 complex entries = 64 (RIS elements, ULA) x 16 (subcarriers),
  flattened element-major (E:67/E:275 comment "64 * 16 * 2");
* pilots ``Yp`` have ``Pilot_num`` complex entries: a comb over the (element,
  subcarrier) grid -- 16 elements (stride 4) x 8 subcarriers (stride 2) for P128 --
  so pilot ``p`` sits at grid cell ``(p // 8, p % 8)`` exactly as the reference's
  row-major reshape to (2, 16, 8) assumes (R:108);
* ``Hlabel`` is the full-grid LS estimate ``H + n_LS``; the LS noise gain is
  calibrated so NMSE_LS(dB) = 2.85 - SNR(dB), the line read off the reference
  figure (BASELINE.md "Derived calibration targets");
* ``Hperf`` is the noiseless channel.

Propagation: multipath H[m, f] = sum_p a_p e^{-j pi m sin(theta_p)} e^{-j 2 pi f tau_p / 16},
per-sample normalised to unit mean power.  Default model ("geometric"): like a ray-traced
DeepMIMO scene, each scenario has a FIXED environment -- its scatterers (each a cluster of
sub-rays) sit at fixed angles of arrival / excess delays at the RIS (small jitter for position
dependence), scenario 0 adds a LoS ray (Rician K = 6 dB), scenarios 1 and 2 share two
scatterers and a fraction of their samples has the scenario-specific scatterers blocked, which
makes those samples genuinely ambiguous for the scenario classifier (the reference's SC
accuracy saturates near 0.945).  The 3 users of a scenario are statistically alike (the
reference's per-stream BatchNorm punishes users with different statistics, see README);
path phases and +-10% amplitudes are random per sample.  Knobs: ``GEO``.
The alternative "cluster" model (v1: random cluster centre / spread / delays per sample) is
kept for comparison: its best linear estimator from the pilots only reaches ~-1.5 dB NMSE
(see reports/r1_gen_v1), i.e. it is not learnable from 128 pilots.
Everything is vectorised torch, so it runs on the GPU (HBM-resident datasets are generated
in place) or on the CPU.
"""
from __future__ import annotations

import hashlib
import math
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

N_ELEM = 64
N_SUBC = 16
H_DIM = N_ELEM * N_SUBC  # 1024
LS_GAIN_DB = 2.85        # NMSE_LS(dB) = LS_GAIN_DB - SNR(dB)


@dataclass(frozen=True)
class ScenarioSpec:
    n_paths: int
    k_factor_db: Optional[float]  # Rician K of the LoS path; None = NLoS
    angle_spread_deg: float
    max_delay: float              # tau in units of 1/(N_SUBC * df); phase = 2 pi f tau / N_SUBC
    decay: float                  # power-delay-profile decay constant (same units)


SCENARIOS: Dict[int, ScenarioSpec] = {
    0: ScenarioSpec(n_paths=3, k_factor_db=6.0, angle_spread_deg=6.0, max_delay=2.0, decay=1.5),
    1: ScenarioSpec(n_paths=6, k_factor_db=None, angle_spread_deg=14.0, max_delay=4.0, decay=2.5),
    2: ScenarioSpec(n_paths=10, k_factor_db=None, angle_spread_deg=28.0, max_delay=6.0, decay=4.0),
}
USER_MEAN_ANGLE_DEG = {0: -25.0, 1: 5.0, 2: 30.0}
USER_ANGLE_JITTER_DEG = 12.0


@dataclass(frozen=True)
class GeoScenario:
    los: bool
    k_factor_db: float
    angles_deg: tuple      # scenario-specific scatterers (AoA at the RIS)
    delays: tuple          # their excess delays (units: 1/16 of the OFDM symbol)
    powers_db: tuple
    shared: bool           # also sees the shared scatterers SHARED_*


GEO_SCENARIOS: Dict[int, GeoScenario] = {
    0: GeoScenario(True, 6.0, (-40.0, 35.0), (1.5, 2.5), (0.0, -3.0), False),
    1: GeoScenario(False, 0.0, (-55.0, 50.0), (0.5, 3.5), (0.0, -2.0), True),
    2: GeoScenario(False, 0.0, (-60.0, -35.0, 5.0, 45.0), (0.3, 1.0, 3.4, 4.2), (0.0, -1.0, -2.0, -3.0), True),
}
SHARED_ANGLES_DEG = (-10.0, 20.0)
SHARED_DELAYS = (1.5, 2.5)
SHARED_POWERS_DB = (-2.0, -3.0)
# Knobs of the geometric model (defaults = v3).  Sub-paths: every scatterer is a small cluster of
# ``n_sub`` rays at fixed offsets (drawn once per (scenario, user, scatterer), spread
# ``sub_spread_deg`` / ``sub_delay_spread``), each with its own random phase per sample -- more
# degrees of freedom per user, like the many rays of a ray-traced scene.  ``user_drift_deg``: per
# sample, ALL angles of a user shift together by U(-1, 1) * drift (position along the user row).
# ``user_los_deg``: LoS angle of each user (scenario 0); ``user_tilt_db``: how strongly a user's
# position re-weights the scatterers.  Users whose statistics differ a lot interact badly with the
# reference's per-stream BatchNorm (train-mode statistics per user vs one running average at eval).
# Defaults = the calibrated "v5c" scene (scripts/gen_sweep.py; reports/r1_gen_v5): 8 sub-rays per
# scatterer, statistically alike users, 16% of the scenario-1/2 samples blocked down to the shared
# scatterers (ambiguous between those scenarios), scenario-specific scatterers 10 dB below the
# shared ones.  GEO_V3 keeps the first geometric calibration for comparison.
GEO_V3 = dict(angle_jitter_deg=0.1, delay_jitter=0.01, los_jitter_deg=0.5, block_prob=0.1, block_db=15.0,
              n_sub=1, sub_spread_deg=0.0, sub_delay_spread=0.0, user_drift_deg=0.0, amp_jitter=0.1,
              user_tilt_db=3.0, user_los_deg=(-25.0, 5.0, 30.0), own_db=0.0)
GEO = dict(GEO_V3, angle_jitter_deg=0.05, block_prob=0.16, block_db=40.0, n_sub=8, sub_spread_deg=3.0,
           sub_delay_spread=0.6, user_tilt_db=0.0, user_los_deg=(-2.0, 0.0, 2.0), own_db=-10.0)
# ``own_db``: power offset of the scenario-specific scatterers of the scenarios that also see the
# shared ones (1, 2): lower = weaker scenario signature, harder classification at low SNR.
CHANNEL_MODEL = "geometric"


def pilot_layout(pilot_num: int) -> Tuple[int, int]:
    """(#elements, #subcarriers) of the pilot comb; Pilot_num = product."""
    if pilot_num == 128:
        return 16, 8
    if pilot_num == 256:
        return 16, 16
    if pilot_num == 64:
        return 8, 8
    raise ValueError(f"unsupported Pilot_num {pilot_num}")


def pilot_indices(pilot_num: int, device=None) -> torch.Tensor:
    """Flat H indices (element*16 + subcarrier) of the pilot comb, pilot-major order."""
    na, nf = pilot_layout(pilot_num)
    ea = torch.arange(na, device=device) * (N_ELEM // na)
    fs = torch.arange(nf, device=device) * (N_SUBC // nf)
    return (ea[:, None] * N_SUBC + fs[None, :]).reshape(-1)


def seed_for(*parts) -> int:
    h = hashlib.sha256("/".join(str(p) for p in parts).encode()).digest()
    return int.from_bytes(h[:8], "little") & ((1 << 62) - 1)


def _gen(seed: int, device) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


def generate_channels(n: int, scenario: int, user: int, seed: int, device="cpu", chunk: int = 8192,
                      model: Optional[str] = None) -> torch.Tensor:
    """(n, 1024) complex64 perfect channels of one (scenario, user) stream."""
    if (model or CHANNEL_MODEL) == "geometric":
        return generate_channels_geometric(n, scenario, user, seed, device, chunk)
    return generate_channels_cluster(n, scenario, user, seed, device, chunk)


def _steer(amp_phase: torch.Tensor, ang_deg: torch.Tensor, tau: torch.Tensor, device) -> torch.Tensor:
    b, P = ang_deg.shape
    m = torch.arange(N_ELEM, device=device, dtype=torch.float32)
    f = torch.arange(N_SUBC, device=device, dtype=torch.float32)
    sv = torch.polar(torch.ones(b, P, N_ELEM, device=device), -math.pi * m * torch.sin(torch.deg2rad(ang_deg))[..., None])
    fv = torch.polar(torch.ones(b, P, N_SUBC, device=device), -2 * math.pi * f * tau[..., None] / N_SUBC)
    H = torch.einsum("bp,bpm,bpf->bmf", amp_phase, sv, fv).reshape(b, H_DIM)
    return H / torch.sqrt((H.abs() ** 2).mean(dim=1, keepdim=True))


def generate_channels_geometric(n: int, scenario: int, user: int, seed: int, device="cpu",
                                chunk: int = 8192) -> torch.Tensor:
    """Fixed-environment model (module docstring; knobs in ``GEO``)."""
    spec = GEO_SCENARIOS[scenario]
    cfg = GEO
    device = torch.device(device)
    g = _gen(seed, device)
    angs, dls, pws = list(spec.angles_deg), list(spec.delays), list(spec.powers_db)
    n_own = len(angs)
    if spec.shared:
        pws = [p + cfg["own_db"] for p in pws]
        angs += list(SHARED_ANGLES_DEG)
        dls += list(SHARED_DELAYS)
        pws += list(SHARED_POWERS_DB)
    K = len(angs)
    # user-dependent visibility of the scatterers
    upw = torch.tensor(pws, device=device) - cfg["user_tilt_db"] * (
        torch.arange(K, device=device) - user * (K - 1) / 2).abs() / max(K - 1, 1)
    # fixed sub-ray geometry: a property of each scatterer (the shared scatterers look the same from
    # every scenario that sees them), not of the sample
    ns = int(cfg["n_sub"])
    sub_a = torch.zeros(K, ns)
    sub_d = torch.zeros(K, ns)
    if ns > 1:
        for j in range(K):
            key = ("geo-sub", scenario, j) if j < n_own else ("geo-sub-shared", j - n_own)
            gs = _gen(seed_for(*key), torch.device("cpu"))
            sub_a[j] = cfg["sub_spread_deg"] * torch.randn(ns, generator=gs)
            sub_d[j] = cfg["sub_delay_spread"] * torch.rand(ns, generator=gs)
    sub_a, sub_d = sub_a.to(device), sub_d.to(device)
    out = torch.empty(n, H_DIM, dtype=torch.complex64, device=device)
    base_a = torch.tensor(angs, device=device)
    base_d = torch.tensor(dls, device=device)
    for s in range(0, n, chunk):
        b = min(chunk, n - s)
        drift = cfg["user_drift_deg"] * (2 * torch.rand(b, 1, generator=g, device=device) - 1)
        ang = base_a.repeat(b, 1) + cfg["angle_jitter_deg"] * torch.randn(b, K, generator=g, device=device) + drift
        tau = base_d.repeat(b, 1) + cfg["delay_jitter"] * torch.rand(b, K, generator=g, device=device)
        pw = (10 ** (upw / 10)).repeat(b, 1)
        if spec.shared and cfg["block_prob"] > 0:
            blk = torch.rand(b, 1, generator=g, device=device) < cfg["block_prob"]
            att = torch.ones(b, K, device=device)
            att[:, :n_own] = 10 ** (-cfg["block_db"] / 10)
            pw = torch.where(blk, pw * att, pw)
        pw = pw / pw.sum(dim=1, keepdim=True)
        amp = torch.sqrt(pw) * (1 + cfg["amp_jitter"] * torch.randn(b, K, generator=g, device=device))
        # expand scatterers into sub-rays (equal power split, independent phases)
        ang = (ang[:, :, None] + sub_a[None]).reshape(b, K * ns)
        tau = (tau[:, :, None] + sub_d[None]).reshape(b, K * ns)
        amp = (amp[:, :, None] / math.sqrt(ns)).expand(b, K, ns).reshape(b, K * ns)
        ph = 2 * math.pi * torch.rand(b, K * ns, generator=g, device=device)
        if spec.los:
            Kf = 10 ** (spec.k_factor_db / 10)
            la = cfg["user_los_deg"][user] + cfg["los_jitter_deg"] * (2 * torch.rand(b, 1, generator=g, device=device) - 1) + drift
            ld = 0.2 * torch.rand(b, 1, generator=g, device=device)
            ang = torch.cat([la, ang], 1)
            tau = torch.cat([ld, tau], 1)
            amp = torch.cat([torch.full((b, 1), math.sqrt(Kf), device=device), amp], 1)
            ph = torch.cat([2 * math.pi * torch.rand(b, 1, generator=g, device=device), ph], 1)
        out[s:s + b] = _steer(torch.polar(amp, ph), ang, tau, device)
    return out


def generate_channels_cluster(n: int, scenario: int, user: int, seed: int, device="cpu",
                              chunk: int = 8192) -> torch.Tensor:
    """v1 random-cluster model (kept for comparison; not learnable from 128 pilots)."""
    spec = SCENARIOS[scenario]
    device = torch.device(device)
    g = _gen(seed, device)
    out = torch.empty(n, H_DIM, dtype=torch.complex64, device=device)
    m = torch.arange(N_ELEM, device=device, dtype=torch.float32)
    f = torch.arange(N_SUBC, device=device, dtype=torch.float32)
    for s in range(0, n, chunk):
        b = min(chunk, n - s)
        P = spec.n_paths
        mean = math.radians(USER_MEAN_ANGLE_DEG[user])
        centre = mean + math.radians(USER_ANGLE_JITTER_DEG) * (torch.rand(b, 1, generator=g, device=device) * 2 - 1)
        theta = centre + math.radians(spec.angle_spread_deg) * torch.randn(b, P, generator=g, device=device)
        tau = spec.max_delay * torch.rand(b, P, generator=g, device=device)
        power = torch.exp(-tau / spec.decay)
        amp = torch.complex(torch.randn(b, P, generator=g, device=device),
                            torch.randn(b, P, generator=g, device=device)) * math.sqrt(0.5)
        if spec.k_factor_db is not None:
            # path 0 is the LoS ray: deterministic-magnitude, zero delay, at the cluster centre
            K = 10 ** (spec.k_factor_db / 10)
            theta[:, 0] = centre[:, 0]
            tau[:, 0] = 0.0
            power[:, 0] = 1.0
            los_phase = 2 * math.pi * torch.rand(b, generator=g, device=device)
            amp[:, 0] = torch.polar(torch.ones(b, device=device), los_phase)
            nlos = power[:, 1:].sum(1, keepdim=True)
            power[:, 1:] = power[:, 1:] / nlos * (1.0 / K) * power[:, :1]
        amp = amp * torch.sqrt(power)
        sv = torch.polar(torch.ones(b, P, N_ELEM, device=device), -math.pi * m * torch.sin(theta)[..., None])
        fv = torch.polar(torch.ones(b, P, N_SUBC, device=device), -2 * math.pi * f * tau[..., None] / N_SUBC)
        H = torch.einsum("bp,bpm,bpf->bmf", amp, sv, fv).reshape(b, H_DIM)
        H = H / torch.sqrt((H.abs() ** 2).mean(dim=1, keepdim=True))
        out[s:s + b] = H
    return out


def complex_noise(shape, var: float, g: torch.Generator, device) -> torch.Tensor:
    s = math.sqrt(var / 2)
    return torch.complex(torch.randn(shape, generator=g, device=device) * s,
                         torch.randn(shape, generator=g, device=device) * s)


def observe(H: torch.Tensor, pilot_num: int, snr_db: float, seed: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Pilot observations Yp (n, Pilot_num) and the full-grid LS estimate (n, 1024)."""
    device = H.device
    g = _gen(seed, device)
    sigma2 = 10 ** (-snr_db / 10)
    idx = pilot_indices(pilot_num, device)
    Yp = H[:, idx] + complex_noise((H.shape[0], idx.numel()), sigma2, g, device)
    HLS = H + complex_noise(H.shape, sigma2 * 10 ** (LS_GAIN_DB / 10), g, device)
    return Yp, HLS


def generate_stream(n: int, scenario: int, user: int, snr_db: float, pilot_num: int = 128, split: str = "train",
                    base_seed: int = 0, device="cpu"):
    """One (scenario, user) stream: (Yp, Hlabel, Hperf, Indicator) -- reference get_data layout (R:48-73)."""
    H = generate_channels(n, scenario, user, seed_for(base_seed, split, "H", scenario, user), device)
    Yp, HLS = observe(H, pilot_num, snr_db, seed_for(base_seed, split, "obs", scenario, user, snr_db))
    ind = torch.full((n,), scenario, dtype=torch.long, device=device)
    return Yp, HLS, H, ind


def generate_mixed(n: int, snr_db: float, pilot_num: int = 128, index: int = -1, base_seed: int = 0,
                   split: str = "test", device="cpu"):
    """Mixed-scenario test set (index=-1: all scenarios/users uniformly, Test.py:127-129)."""
    device = torch.device(device)
    g = _gen(seed_for(base_seed, split, "mix", n, index), device)
    if index >= 0:
        scen = torch.full((n,), index, dtype=torch.long, device=device)
    else:
        scen = torch.randint(0, len(SCENARIOS), (n,), generator=g, device=device)
    users = torch.randint(0, len(USER_MEAN_ANGLE_DEG), (n,), generator=g, device=device)
    H = torch.empty(n, H_DIM, dtype=torch.complex64, device=device)
    for s in SCENARIOS:
        for u in USER_MEAN_ANGLE_DEG:
            sel = ((scen == s) & (users == u)).nonzero().flatten()
            if sel.numel():
                H[sel] = generate_channels(sel.numel(), s, u, seed_for(base_seed, split, "H", s, u, n), device)
    Yp, HLS = observe(H, pilot_num, snr_db, seed_for(base_seed, split, "obs", snr_db, n))
    return Yp, HLS, H, scen


# ----------------------------------------------------------------------------- packing
def pack_pilots(Yp: torch.Tensor, pilot_num: int = 128) -> torch.Tensor:
    """complex (B, P) -> real (B, 2, Ha, Wf): all real parts then all imaginary parts (R:108)."""
    na, nf = pilot_layout(pilot_num)
    return torch.cat([Yp.real, Yp.imag], dim=1).float().reshape(Yp.shape[0], 2, na, nf)


def pack_channel(H: torch.Tensor) -> torch.Tensor:
    """complex (B, 1024) -> real (B, 2048) = [Re | Im] (R:104)."""
    return torch.cat([H.real, H.imag], dim=1).float()


def unpack_channel(Hr: torch.Tensor) -> torch.Tensor:
    d = Hr.shape[1] // 2
    return torch.complex(Hr[:, :d].float(), Hr[:, d:].float())
