"""HDCE weight averaging (RunnerConfig.swa_epochs, the FIG1 high-SNR option): the "swa" checkpoint holds the mean
of the last epochs' weights with BN statistics re-estimated on the training streams, the trained model is left
as it was, and model_val(hdce_tag="swa") evaluates it (CPU, deterministic)."""
import os

import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import Conv_P128, SC_P128
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train import checkpoint as ck
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.evaluate import model_val, recalibrate_bn
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.runner import Y2HRunner


def _train(tmp_path, name, epochs, swa):
    ws = str(tmp_path / name)
    r = Y2HRunner(n_epochs=epochs, swa_epochs=swa, data_len=60, batch_size_DML=16, device="cpu", workspace=ws,
                  data_dir=str(tmp_path / "data"), print_freq=1000)
    torch.manual_seed(0)
    r.train_Conv_Linear_of_HDCE()
    return r, ck.ckpt_dir(ws, 128, make=False)


def _load(d, name, tag):
    key = "conv" if name.startswith("Conv") else "linear"
    return torch.load(os.path.join(d, f"{name}_16_10dB_{tag}_DML.pth"), weights_only=True)[key]


def _is_bn_stat(k):
    return k.endswith(("running_mean", "running_var", "num_batches_tracked"))


def test_swa_is_the_mean_of_the_epoch_snapshots(tmp_path):
    _, d2 = _train(tmp_path, "two", 2, 1)     # epochs 0-1: its final weights are the 3-epoch run's epoch-1 snapshot
    r3, d3 = _train(tmp_path, "three", 3, 2)
    for name in ("Conv0", "Conv1", "Conv2", "Linear"):
        w1, w2, avg = _load(d2, name, "epoch1"), _load(d3, name, "epoch2"), _load(d3, name, "swa")
        one = _load(d2, name, "swa")
        for k in avg:
            if _is_bn_stat(k):
                continue
            assert torch.equal(one[k], w1[k]), k                       # swa_epochs=1: the last epoch's weights
            assert torch.allclose(avg[k], (w1[k] + w2[k]) / 2, atol=1e-7, rtol=0), (name, k)
    # the trained model keeps its own weights and statistics: the epoch-2 checkpoint was saved before the average,
    # and the model after training still matches it
    for e, conv in enumerate(r3.hdce_model.convs):
        sd = _load(d3, f"Conv{e}", "epoch2")
        for k, v in conv.state_dict().items():
            assert torch.equal(v, sd["module." + k]), (e, k)


def test_swa_bn_statistics_are_reestimated_on_the_training_streams(tmp_path):
    r, d = _train(tmp_path, "one", 2, 1)
    tr, _ = r.device_stores()
    convs = [Conv_P128(128) for _ in range(3)]
    for e, c in enumerate(convs):
        c.load_state_dict({k[len("module."):]: v for k, v in _load(d, f"Conv{e}", "swa").items()})
    xs, ex = [], []
    for e in range(3):
        Yp = tr.Yp.index_select(0, (tr.scen == e).nonzero().flatten())
        xs.append(Yp.transpose(0, 1).reshape(-1, *Yp.shape[2:]))
        ex.append(torch.full((xs[-1].shape[0],), e))
    want = [[m.running_var.clone() for m in c.modules() if isinstance(m, torch.nn.BatchNorm2d)] for c in convs]
    for c, w in zip(convs, want):   # (the loaded statistics are the saved ones)
        bns = [m for m in c.modules() if isinstance(m, torch.nn.BatchNorm2d)]
        for m in bns:
            m.running_var.fill_(7.0)
    recalibrate_bn(convs, torch.cat(xs), torch.cat(ex), chunk=3 * 16)
    for c, w in zip(convs, want):
        got = [m.running_var for m in c.modules() if isinstance(m, torch.nn.BatchNorm2d)]
        for a, b in zip(got, w):
            assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)
    epoch = _load(d, "Conv0", "epoch1")
    swa = _load(d, "Conv0", "swa")
    assert not torch.equal(epoch["module.cnn.1.running_var"], swa["module.cnn.1.running_var"])
    # model_val evaluates the average through hdce_tag (the classifiers keep their epoch tag)
    torch.save({"cnn": SC_P128(128).state_dict()}, os.path.join(d, "16_10dB_epoch1_DML_SC.pth"))
    mv = model_val(device="cpu", workspace=r.workspace, batch_size_DML=16, training_data_len=60, hdce_tag="swa")
    mv.epoch_tag = "epoch1"
    _, _, loaded, _ = mv.load_models()
    for k, v in loaded[0].state_dict().items():
        assert torch.equal(v, swa["module." + k]), k
