"""model_val's per-SNR evaluation on the CPU (torch path): baselines, routing, test-time BN adaptation."""
import math

import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import (Conv_P128, FC_P128,
                                                                                               SC_P128)
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.evaluate import (model_val,
                                                                                           recalibrate_bn, restore_bn)


def _models():
    torch.manual_seed(0)
    convs = [Conv_P128(128).eval() for _ in range(3)]
    return SC_P128(128).eval(), convs, FC_P128(128).eval()


def test_recalibrate_and_restore_bn_roundtrip():
    _, convs, _ = _models()
    before = [{k: v.clone() for k, v in c.state_dict().items()} for c in convs]
    x = torch.randn(64, 2, 16, 8) * 3 + 1
    expert = torch.arange(64) % 3
    saved = recalibrate_bn(convs, x, expert)
    bn = [m for m in convs[1].modules() if isinstance(m, torch.nn.BatchNorm2d)][0]
    assert not torch.allclose(bn.running_var, before[1][[k for k in before[1] if k.endswith("running_var")][0]])
    assert all(not c.training for c in convs)
    restore_bn(convs, saved)
    for c, b in zip(convs, before):
        for k, v in c.state_dict().items():
            assert torch.equal(v, b[k]), k


def test_evaluate_snr_reports_both_mmse_rows_and_bn_adapt():
    sc, convs, fc = _models()
    mv = model_val(device="cpu", data_len_for_test=300)
    r = mv.evaluate_snr(10.0, sc, None, convs, fc)
    db = lambda v: 10 * math.log10(v)
    assert abs(db(r["nmse_ls"]) - (2.85 - 10)) < 0.3
    assert db(r["nmse_lmmse"]) < db(r["nmse_mmse"]) < db(r["nmse_ls"])
    assert math.isnan(r["nmse_quantum"]) and 0.0 <= r["acc_classical"] <= 1.0
    state = [{k: v.clone() for k, v in c.state_dict().items()} for c in convs]
    mva = model_val(device="cpu", data_len_for_test=300, bn_adapt=True)
    ra = mva.evaluate_snr(10.0, sc, None, convs, fc)
    assert ra["nmse_classical"] != r["nmse_classical"] and ra["nmse_ls"] == r["nmse_ls"]
    for c, s in zip(convs, state):   # adaptation is scoped to the evaluation
        for k, v in c.state_dict().items():
            assert torch.equal(v, s[k]), k
