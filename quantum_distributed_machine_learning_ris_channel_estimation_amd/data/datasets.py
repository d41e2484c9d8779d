"""Datasets: reference-compatible host datasets and the HBM-resident 9-stream store.

Reference: ``Y2HRunner.get_data`` (R:48-73) loads
``available_data/{Yp|Hlabel|Hperf}{s}_{P}_1024_{SNR}dB_{u}_datalen_{N}.npy``, truncates,
and splits sequentially at ``train_test_ratio``; ``get_dataloader_DML`` (R:75-95) zips
the 9 (scenario, user) streams into ``generate_data.DatasetFolder_DML`` whose item i is
the 9-list of ``[Yp[i], Hlabel[i], Hperf[i], Indicator[i]]`` (R:181-182).  ``Test.py``
additionally uses ``DatasetFolder(td)`` over a ``generate_datapair`` tuple (T:127-140).

MI355X design: the training path never goes through a host DataLoader.  All 9
streams are packed once into device tensors (``DMLStore``): pilots as (S, N, 2, H, W)
real images, labels as (S, N, 2048) [Re|Im] -- ~3 GB at the reference size, trivial
for 288 GB of HBM -- and a step gathers its rows by index on the device.  The host
datasets below exist for API compatibility and tests.
"""
from __future__ import annotations

import os
import warnings
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

from .channel import generate_mixed, generate_stream, pack_channel, pack_pilots


def npy_name(kind: str, scenario: int, pilot_num: int, snr_db: int, user: int, data_len: int) -> str:
    return f"{kind}{scenario}_{pilot_num}_1024_{snr_db}dB_{user}_datalen_{data_len}.npy"


class DatasetFolder_DML(Dataset):
    """Zip of per-stream ``[Yp, Hlabel, Hperf, Indicator]`` arrays (reference usage R:87, R:181)."""

    def __init__(self, *streams: Sequence):
        if not streams:
            raise ValueError("need at least one stream")
        self.streams = [[_as_tensor(a) for a in s] for s in streams]
        self.n = min(len(s[0]) for s in self.streams)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return [[a[i] for a in s] for s in self.streams]


class DatasetFolder(Dataset):
    """Single-stream dataset over ``(Yp, HLS, Hperfect, indicator)`` (Test.py:130, T:140)."""

    def __init__(self, td: Sequence):
        self.td = [_as_tensor(a) for a in td]

    def __len__(self):
        return len(self.td[0])

    def __getitem__(self, i):
        return tuple(a[i] for a in self.td)


def _as_tensor(a):
    if isinstance(a, torch.Tensor):
        return a
    return torch.from_numpy(np.ascontiguousarray(a))


def generate_datapair(Ns: int, Pilot_num: int = 128, index: int = -1, SNRdb: float = 10, start: int = 0,
                      training_data_len: int = 20000, base_seed: int = 0, device="cpu"):
    """Test data at an arbitrary SNR (Test.py:127-129).  ``start`` keys a split disjoint from
    training; returns numpy complex arrays ``(Yp, HLS, Hperfect, indicator)``."""
    Yp, HLS, H, ind = generate_mixed(Ns, SNRdb, Pilot_num, index, base_seed=base_seed,
                                     split=f"test@{start}/{training_data_len}", device=device)
    return Yp.cpu().numpy(), HLS.cpu().numpy(), H.cpu().numpy(), ind.cpu().numpy()


def stream_paths(data_dir: str, scenario: int, user: int, pilot_num: int, snr_db: int, data_len: int) -> List[str]:
    return [os.path.join(data_dir, npy_name(k, scenario, pilot_num, snr_db, user, data_len))
            for k in ("Yp", "Hlabel", "Hperf")]


def load_or_generate_stream(data_dir: str, scenario: int, user: int, pilot_num: int, snr_db: int, data_len: int,
                            synthetic: bool = True, base_seed: int = 0, device="cpu"):
    """Reference .npy file pattern when present, else the synthetic generator."""
    paths = stream_paths(data_dir, scenario, user, pilot_num, snr_db, data_len)
    if all(os.path.exists(p) for p in paths):
        Yp, HL, HP = (torch.from_numpy(np.load(p)).to(device) for p in paths)  # allow_pickle=False (default)
        n = min(len(Yp), data_len)
        ind = torch.full((n,), scenario, dtype=torch.long, device=device)
        return Yp[:n].to(torch.complex64), HL[:n].to(torch.complex64), HP[:n].to(torch.complex64), ind
    if not synthetic:
        raise FileNotFoundError(paths[0])
    return generate_stream(data_len, scenario, user, snr_db, pilot_num, "train", base_seed, device)


def save_stream_npy(data_dir: str, stream, scenario: int, user: int, pilot_num: int, snr_db: int,
                    data_len: int) -> None:
    os.makedirs(data_dir, exist_ok=True)
    for kind, arr in zip(("Yp", "Hlabel", "Hperf"), stream[:3]):
        np.save(os.path.join(data_dir, npy_name(kind, scenario, pilot_num, snr_db, user, data_len)),
                arr.cpu().numpy())


def split_stream(stream, ratio: float):
    """Sequential split at ``int(N * ratio)`` (R:67-71)."""
    n = stream[0].shape[0]
    s = int(n * ratio)
    return [a[:s] for a in stream], [a[s:] for a in stream]


@dataclass
class DMLStore:
    """Device-resident packed 9-stream data: pilots (S,N,2,H,W), labels (S,N,2048)."""
    Yp: torch.Tensor
    Hlabel: torch.Tensor
    Hperf: torch.Tensor
    scen: torch.Tensor        # (S,) scenario id of each stream
    user: torch.Tensor        # (S,) user id of each stream

    @property
    def n(self) -> int:
        return self.Yp.shape[1]

    @property
    def n_streams(self) -> int:
        return self.Yp.shape[0]

    def to(self, device, label_dtype=None) -> "DMLStore":
        ld = label_dtype
        return DMLStore(self.Yp.to(device), self.Hlabel.to(device, ld) if ld else self.Hlabel.to(device),
                        self.Hperf.to(device, ld) if ld else self.Hperf.to(device),
                        self.scen.to(device), self.user.to(device))

    def shard(self, rank: int, world: int, drop_remainder: bool = True) -> "DMLStore":
        """Contiguous per-rank shard of the sample axis (distributed DML sampler).  Training shards are
        equal (``drop_remainder``: every rank runs the same number of lock-step batches); validation
        shards (``drop_remainder=False``) cover every sample, the first ``n % world`` ranks one more."""
        per, rem = divmod(self.n, world)
        if drop_remainder:
            s = slice(rank * per, (rank + 1) * per)
        else:
            lo = rank * per + min(rank, rem)
            s = slice(lo, lo + per + (rank < rem))
        return DMLStore(self.Yp[:, s], self.Hlabel[:, s], self.Hperf[:, s], self.scen, self.user)

    def gather(self, idx: torch.Tensor):
        """Rows ``idx`` (B,) of every stream -> (S,B,2,H,W), (S,B,2048), (S,B,2048)."""
        return (self.Yp.index_select(1, idx), self.Hlabel.index_select(1, idx), self.Hperf.index_select(1, idx))


def build_store(streams: List, scen_ids: List[int], user_ids: List[int], pilot_num: int, device,
                label_dtype=torch.float32) -> DMLStore:
    Yp = torch.stack([pack_pilots(s[0].to(device), pilot_num) for s in streams])
    HL = torch.stack([pack_channel(s[1].to(device)).to(label_dtype) for s in streams])
    HP = torch.stack([pack_channel(s[2].to(device)).to(label_dtype) for s in streams])
    return DMLStore(Yp, HL, HP, torch.tensor(scen_ids, device=device), torch.tensor(user_ids, device=device))


def make_dml_stores(data_len: int, pilot_num: int, snr_db: int, ratio: float, device, data_dir: str = "available_data",
                    synthetic: bool = True, base_seed: int = 0, n_scenarios: int = 3, n_users: int = 3,
                    label_dtype=torch.float32) -> Tuple[DMLStore, DMLStore]:
    """Train / val stores for all (scenario, user) streams in reference order (R:76-84).

    Real data (the reference's 27 .npy files under ``data_dir``) is all-or-nothing: some streams on
    disk and others missing is an error (never a silent real/synthetic mix), and falling back to the
    synthetic generator is announced with a warning unless ``data_dir`` is None (synthetic by intent)."""
    if data_dir is not None:
        have = [all(os.path.exists(p) for p in stream_paths(data_dir, s, u, pilot_num, snr_db, data_len))
                for s in range(n_scenarios) for u in range(n_users)]
        if any(have) and not all(have):
            missing = [i for i, h in enumerate(have) if not h]
            raise FileNotFoundError(f"{data_dir}: data files for streams {missing} (scenario*{n_users}+user) are "
                                    f"missing while the others exist; refusing to mix real and synthetic data")
        if not any(have):
            if not synthetic:
                raise FileNotFoundError(stream_paths(data_dir, 0, 0, pilot_num, snr_db, data_len)[0])
            warnings.warn(f"no reference data files under {data_dir!r}: using the synthetic DeepMIMO-shaped "
                          "generator for all streams", stacklevel=2)
    else:
        data_dir = ""
    tr, va, sids, uids = [], [], [], []
    for s in range(n_scenarios):
        for u in range(n_users):
            st = load_or_generate_stream(data_dir, s, u, pilot_num, snr_db, data_len, synthetic, base_seed, device)
            a, b = split_stream(st, ratio)
            tr.append(a)
            va.append(b)
            sids.append(s)
            uids.append(u)
    return (build_store(tr, sids, uids, pilot_num, device, label_dtype),
            build_store(va, sids, uids, pilot_num, device, label_dtype))
