"""Y2HRunner training on the GPU: a graphed epoch (one HIP graph per full batch, captured after warm-up
steps whose effects _capture_preserving rolls back) ends bit-identical to the same epoch run eagerly --
weights, optimizer moments, the optimizer-written bf16 FC shadow, BN running statistics and
num_batches_tracked (the snapshot must cover every tensor a step mutates)."""
import warnings

import pytest
import torch

pytestmark = pytest.mark.gpu


def _train_hdce(tmp_path, graphs: bool):
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.runner import Y2HRunner
    r = Y2HRunner()
    for k, v in dict(device="cuda", n_epochs=2, data_len=200, batch_size_DML=16, print_freq=1000,
                     workspace=str(tmp_path / ("g" if graphs else "e")), data_dir=str(tmp_path / "nodata"),
                     hip_graphs=graphs, seed=0).items():
        setattr(r, k, v)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")   # (synthetic-data notice)
        m = r.train_Conv_Linear_of_HDCE()
    torch.cuda.synchronize()
    return r, m


def test_graphed_hdce_epochs_match_eager(tmp_path):
    rg, mg = _train_hdce(tmp_path, True)
    re_, me = _train_hdce(tmp_path, False)
    assert torch.equal(mg.space.flat, me.space.flat)
    if mg.fc_shadow is not None:
        assert torch.equal(mg.fc_shadow, me.fc_shadow)
    for a, b in zip(mg.run_mean + mg.run_var + list(mg.nbt), me.run_mean + me.run_var + list(me.nbt)):
        assert torch.equal(a, b)
    assert rg.train_HDCE_losses == re_.train_HDCE_losses and rg.val_HDCE_nmse == re_.val_HDCE_nmse
