"""Reference entry points and the CLI."""
import importlib
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_module_names_import():
    est = importlib.import_module("Estimators_QuantumNAT_onchipQNN")
    for name in ("DCE_P128", "SC_P128", "QSC_P128", "Conv_P128", "FC_P128", "NMSE_cuda", "NMSELoss"):
        assert hasattr(est, name)
    assert hasattr(importlib.import_module("Estimators"), "Conv_P128")
    assert hasattr(importlib.import_module("Runner_P128"), "OptimizedQSC_P128")
    run = importlib.import_module("Runner_P128_QuantumNAT_onchipQNN")
    r = run.Y2HRunner()
    for k, v in dict(Pilot_num=128, data_len=20000, SNRdb=10, num_workers=0, batch_size=256, batch_size_DML=256,
                     lr=1e-3, lr_decay=30, lr_threshold=1e-6, n_epochs=100, print_freq=50, optimizer="adam",
                     train_test_ratio=0.9).items():
        assert getattr(r, k) == v, k
    assert r.train_QSC_losses == [] and r.val_QSC_losses == [] and r.val_QSC_accuracies == []
    gd = importlib.import_module("generate_data")
    for name in ("DatasetFolder_DML", "DatasetFolder", "generate_datapair", "generate_MMSE_estimate"):
        assert hasattr(gd, name)
    mv = importlib.import_module("Test").model_val()
    assert (mv.training_SNRdb, mv.batch_size, mv.data_len_for_test, mv.indicator) == (10, 200, 10000, -1)


def test_get_optimizer_semantics():
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.runner import Y2HRunner
    r = Y2HRunner()
    p = [torch.nn.Parameter(torch.zeros(2))]
    assert isinstance(r.get_optimizer(p, 1e-3), torch.optim.Adam)
    r.optimizer = "sgd"
    o = r.get_optimizer(p, 1e-3)
    assert isinstance(o, torch.optim.SGD) and o.param_groups[0]["momentum"] == 0.9
    r.optimizer = "rmsprop"
    try:
        r.get_optimizer(p, 1e-3)
        assert False
    except NotImplementedError:
        pass


def test_cli_gen_data(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "quantum_distributed_machine_learning_ris_channel_estimation_amd",
                        "gen-data", "--set", "data_len=20", "--set", f"data_dir={tmp_path}"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    assert len([f for f in os.listdir(tmp_path) if f.endswith(".npy")]) == 27
