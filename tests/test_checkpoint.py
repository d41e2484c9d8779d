"""Reference-compatible checkpoint names, keys, prefixes; safe loading; Test.py-style loader."""
import os

import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import (
    Conv_P128, FC_P128, QSC_P128, SC_P128)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train import checkpoint as ck


def test_hdce_layout_and_prefix(tmp_path):
    d = ck.ckpt_dir(str(tmp_path), 128)
    convs = [Conv_P128() for _ in range(3)]
    fc = FC_P128()
    ck.save_hdce(d, convs, fc, 256, 10, "epoch99")
    for s in range(3):
        p = os.path.join(d, f"Conv{s}_256_10dB_epoch99_DML.pth")
        sd = torch.load(p, weights_only=True)["conv"]
        assert all(k.startswith("module.") for k in sd)
        assert "module.cnn.7.num_batches_tracked" in sd
    sd = torch.load(os.path.join(d, "Linear_256_10dB_epoch99_DML.pth"), weights_only=True)["linear"]
    assert set(sd) == {"module.FC.weight", "module.FC.bias"}
    # Test.py-style loader strips the prefix for an unwrapped model
    c = Conv_P128()
    ck.load_model_state_dict(c, os.path.join(d, "Conv1_256_10dB_epoch99_DML.pth"), "conv", verbose=False)
    assert torch.equal(c.cnn[0].weight, convs[1].cnn[0].weight)


def test_qsc_and_sc_layout(tmp_path):
    d = ck.ckpt_dir(str(tmp_path), 128)
    q = QSC_P128(n_qubits=4)
    ck.save_qsc(d, q, 256, 10, "best", alias=True)
    sd = torch.load(os.path.join(d, "QSC_OPT_256_10dB_best_DML.pth"), weights_only=True)
    assert list(sd)[0] == "qlayer.weights" and not any(k.startswith("module.") for k in sd)
    alias = torch.load(os.path.join(d, "QSC_optimized_best.pth"), weights_only=True)
    assert alias["qsc_config"]["n_qubits"] == 4
    q2 = QSC_P128(n_qubits=4)
    ck.load_model_state_dict(q2, os.path.join(d, "QSC_optimized_best.pth"), "model_state_dict", verbose=False)
    assert torch.equal(q2.qlayer.weights, q.qlayer.weights)
    sc = SC_P128()
    ck.save_sc(d, sc, 256, 10, "epoch99")
    wrapped = torch.nn.DataParallel(SC_P128())  # prefix added back for a wrapped model (T:49-55)
    ck.load_model_state_dict(wrapped, os.path.join(d, "256_10dB_epoch99_DML_SC.pth"), "cnn", verbose=False)
    assert torch.equal(wrapped.module.conv1.weight, sc.conv1.weight)


def test_flat_views_saved_as_plain_tensors(tmp_path):
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel
    m = HDCEModel(128, "cpu", "fp32")
    d = ck.ckpt_dir(str(tmp_path), 128)
    ck.save_hdce(d, m.convs, m.fc, 8, 10, "best")
    size = os.path.getsize(os.path.join(d, "Conv0_8_10dB_best_DML.pth"))
    assert size < 200_000  # a view of the 34 MB flat buffer would have dragged the whole storage along
    ck.save_resume(os.path.join(d, "r.pth"), epoch=3, rng=ck.rng_state(), flat=m.space.flat)
    st = ck.load_resume(os.path.join(d, "r.pth"))
    assert st["epoch"] == 3 and st["flat"].shape == m.space.flat.shape
