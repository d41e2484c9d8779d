"""Synthetic data generator, packing conventions, baselines and dataset plumbing."""
import math
import os

import numpy as np
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.baselines import (
    generate_MMSE_estimate, lmmse_estimate)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.channel import (
    H_DIM, generate_mixed, generate_stream, pack_channel, pack_pilots, pilot_indices, unpack_channel)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.datasets import (
    DatasetFolder, DatasetFolder_DML, generate_datapair, load_or_generate_stream, make_dml_stores, npy_name,
    save_stream_npy, split_stream)


def nmse_db(a, b):
    return 10 * math.log10(float(((a - b).abs() ** 2).sum() / (b.abs() ** 2).sum()))


def test_shapes_and_determinism():
    Yp, HL, HP, ind = generate_stream(50, 1, 2, 10, 128, "train", 0)
    assert Yp.shape == (50, 128) and HL.shape == HP.shape == (50, H_DIM) and Yp.dtype == torch.complex64
    assert (ind == 1).all()
    Yp2, _, _, _ = generate_stream(50, 1, 2, 10, 128, "train", 0)
    assert torch.equal(Yp, Yp2)
    assert abs(float((HP.abs() ** 2).mean()) - 1.0) < 1e-4  # per-sample unit power


def test_ls_calibration_matches_reference_line():
    """NMSE_LS(dB) = 2.85 - SNR, the line read off the reference figure."""
    for snr in (5, 15):
        _, HLS, H, _ = generate_mixed(2000, snr)
        assert abs(nmse_db(HLS, H) - (2.85 - snr)) < 0.1


def test_mmse_improves_on_ls():
    _, HLS, H, _ = generate_mixed(1500, 5.0)
    assert nmse_db(lmmse_estimate(HLS, 10 ** -0.5), H) < nmse_db(HLS, H) - 1.0
    out = generate_MMSE_estimate(HLS.numpy(), 10 ** -0.5)
    assert isinstance(out, np.ndarray) and out.shape == HLS.shape and np.iscomplexobj(out)


def test_subspace_mmse_matches_reference_gap():
    """FIG1's MMSE row sits ~1.4 dB below LS at every SNR: the rank-12 subspace estimator
    lands within 0.3 dB of that at both ends of the sweep, while the Wiener LMMSE gains more."""
    for snr in (5.0, 15.0):
        _, HLS, H, _ = generate_mixed(1500, snr)
        gap = nmse_db(HLS, H) - nmse_db(lmmse_estimate(HLS, 10 ** (-snr / 10), mode="subspace"), H)
        assert abs(gap - 1.4) < 0.3, gap
        assert nmse_db(lmmse_estimate(HLS, 10 ** (-snr / 10)), H) < nmse_db(HLS, H) - 1.4 - 1.0


def test_pilot_grid_layout():
    """pilot p sits at grid cell (p // 8, p % 8) of the packed (2, 16, 8) image (R:108)."""
    idx = pilot_indices(128)
    assert idx.numel() == 128 and idx[1] - idx[0] == 2 and idx[8] - idx[0] == 4 * 16
    Yp = torch.complex(torch.arange(128.).view(1, -1), -torch.arange(128.).view(1, -1))
    img = pack_pilots(Yp)
    assert img.shape == (1, 2, 16, 8)
    assert img[0, 0, 3, 5] == 3 * 8 + 5 and img[0, 1, 3, 5] == -(3 * 8 + 5)
    H = torch.randn(4, 1024, dtype=torch.complex64)
    assert torch.equal(unpack_channel(pack_channel(H)), H)


def test_dataset_folder_dml_items():
    s1 = [np.arange(5), np.arange(5) * 2, np.arange(5) * 3, np.zeros(5)]
    s2 = [np.arange(5) + 10, np.arange(5), np.arange(5), np.ones(5)]
    ds = DatasetFolder_DML(s1, s2)
    item = ds[3]
    assert len(ds) == 5 and len(item) == 2 and [int(v) for v in item[0]] == [3, 6, 9, 0]
    td = generate_datapair(20, 128, -1, 7, start=60000)
    dsf = DatasetFolder(td)
    assert len(dsf) == 20 and len(dsf[0]) == 4


def test_npy_roundtrip_reference_names(tmp_path):
    st = generate_stream(30, 2, 1, 10, 128, "train", 0)
    save_stream_npy(str(tmp_path), st, 2, 1, 128, 10, 30)
    assert os.path.exists(tmp_path / npy_name("Hlabel", 2, 128, 10, 1, 30))
    assert npy_name("Yp", 2, 128, 10, 1, 30) == "Yp2_128_1024_10dB_1_datalen_30.npy"
    back = load_or_generate_stream(str(tmp_path), 2, 1, 128, 10, 30, synthetic=False)
    assert torch.equal(back[0], st[0]) and torch.equal(back[2], st[2])


def test_split_and_stores():
    tr, va = split_stream([torch.arange(10)], 0.9)
    assert tr[0].tolist() == list(range(9)) and va[0].tolist() == [9]
    trs, vas = make_dml_stores(40, 128, 10, 0.9, "cpu")
    assert trs.Yp.shape == (9, 36, 2, 16, 8) and vas.Hlabel.shape == (9, 4, 2048)
    assert trs.scen.tolist() == [0, 0, 0, 1, 1, 1, 2, 2, 2]
    sh = trs.shard(1, 2)
    assert sh.n == 18 and torch.equal(sh.Yp[:, 0], trs.Yp[:, 18])


def test_real_and_synthetic_streams_never_mix(tmp_path):
    """Some reference .npy streams on disk and others missing is an error; none on disk warns."""
    import warnings

    import pytest

    from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.datasets import (
        generate_stream, make_dml_stores, save_stream_npy)
    d = str(tmp_path / "avail")
    save_stream_npy(d, generate_stream(20, 0, 0, 10, 128, "train", 0, "cpu"), 0, 0, 128, 10, 20)
    with pytest.raises(FileNotFoundError, match="mix"):
        make_dml_stores(20, 128, 10, 0.9, "cpu", data_dir=d)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        make_dml_stores(20, 128, 10, 0.9, "cpu", data_dir=str(tmp_path / "none"))
    assert any("synthetic" in str(x.message) for x in w)


def test_val_shards_cover_every_sample():
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.datasets import make_dml_stores
    _, va = make_dml_stores(70, 128, 10, 0.9, "cpu", data_dir=None)   # 7 val samples per stream
    shards = [va.shard(r, 3, drop_remainder=False) for r in range(3)]
    assert sum(s.n for s in shards) == va.n
    import torch
    assert torch.equal(torch.cat([s.Yp for s in shards], 1), va.Yp)
    assert len({va.shard(r, 3).n for r in range(3)}) == 1   # training shards stay equal
