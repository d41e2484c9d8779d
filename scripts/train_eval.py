"""Train the whole system (HDCE estimator, classical SC, quantum SC) and run the NMSE-vs-SNR /
scenario-accuracy sweep; writes results JSON + FIG1/FIG2-style plots.

    python scripts/train_eval.py --epochs 100 --qubits 6 --out reports/
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--qubits", type=int, default=6)
    ap.add_argument("--qml-qubits", default="", help="extra QSC qubit counts for the FIG2 loss curves, e.g. 4,8")
    ap.add_argument("--data-len", type=int, default=20000)
    ap.add_argument("--test-len", type=int, default=10000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default="reports")
    ap.add_argument("--workspace", default="./workspace")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp8"],
                    help="HDCE estimator compute dtype (fp8: e4m3 FC forward GEMM, bf16 convs / backward)")
    ap.add_argument("--hdce-engine", default="hip", choices=["hip", "torch"],
                    help="HDCE training step: the fused HIP kernels, or torch autograd (with --dtype fp32: all fp32)")
    ap.add_argument("--bn-adapt", action="store_true", help="also run the sweep with test-time BN re-estimation "
                    "(written under <out>/bn_adapt)")
    ap.add_argument("--swa-epochs", type=int, default=0, help="also average the HDCE weights over the last K epochs "
                    "and run the sweep on the average (written under <out>/swa, and <out>/swa_bn_adapt with --bn-adapt)")
    a = ap.parse_args()
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.evaluate import model_val
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.runner import Y2HRunner
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.utils.plots import plot_fig2
    os.makedirs(a.out, exist_ok=True)
    common = dict(n_epochs=a.epochs, data_len=a.data_len, batch_size_DML=a.batch, workspace=a.workspace, dtype=a.dtype,
                  hdce_engine=a.hdce_engine, swa_epochs=a.swa_epochs,
                  log_jsonl=os.path.join(a.out, "train_metrics.jsonl"))
    r = Y2HRunner(n_qubits=a.qubits, **common)
    t = {}
    t0 = time.time(); r.train_Conv_Linear_of_HDCE(); t["hdce_s"] = time.time() - t0
    t0 = time.time(); r.train_SC_P128(); t["sc_s"] = time.time() - t0
    curves = {"CNN": list(r.train_SC_losses)}
    extra = [int(q) for q in a.qml_qubits.split(",") if q]
    for q in extra:
        if q == a.qubits:
            continue
        rq = Y2HRunner(n_qubits=q, workspace=os.path.join(a.workspace, f"q{q}"), **{k: v for k, v in common.items() if k != "workspace"})
        rq._stores = r._stores
        t0 = time.time(); rq.train_QSC_P128(); t[f"qsc{q}_s"] = time.time() - t0
        curves[f"QML {q} bits"] = list(rq.train_QSC_losses)
    t0 = time.time(); r.train_QSC_P128(); t[f"qsc{a.qubits}_s"] = time.time() - t0
    curves[f"QML {a.qubits} bits"] = list(r.train_QSC_losses)
    hist = {"train_seconds": t, "loss_curves": curves, "val_QSC_accuracies": r.val_QSC_accuracies,
            "val_SC_accuracies": r.val_SC_accuracies, "val_HDCE_nmse": r.val_HDCE_nmse,
            "train_HDCE_losses": r.train_HDCE_losses}
    with open(os.path.join(a.out, "training_history.json"), "w") as f:
        json.dump(hist, f, indent=1)
    plot_fig2(curves, os.path.join(a.out, "loss_curve.png"))
    mv = model_val(workspace=a.workspace, results_dir=a.out, data_len_for_test=a.test_len,
                   training_data_len=a.data_len, batch_size_DML=a.batch, n_qubits=a.qubits)
    mv.epoch_tag = f"epoch{a.epochs - 1}"
    t0 = time.time()
    mv.test_for_CE_P128_for_all_scenarios()
    t["eval_s"] = time.time() - t0
    if a.bn_adapt:
        mva = model_val(workspace=a.workspace, results_dir=os.path.join(a.out, "bn_adapt"), data_len_for_test=a.test_len,
                        training_data_len=a.data_len, batch_size_DML=a.batch, n_qubits=a.qubits, bn_adapt=True)
        mva.epoch_tag = mv.epoch_tag
        t0 = time.time()
        mva.test_for_CE_P128_for_all_scenarios()
        t["eval_bn_adapt_s"] = time.time() - t0
    if a.swa_epochs > 0:
        for sub, bn in (("swa", False),) + ((("swa_bn_adapt", True),) if a.bn_adapt else ()):
            mvs = model_val(workspace=a.workspace, results_dir=os.path.join(a.out, sub), data_len_for_test=a.test_len,
                            training_data_len=a.data_len, batch_size_DML=a.batch, n_qubits=a.qubits, bn_adapt=bn,
                            hdce_tag="swa")
            mvs.epoch_tag = mv.epoch_tag
            t0 = time.time()
            mvs.test_for_CE_P128_for_all_scenarios()
            t[f"eval_{sub}_s"] = time.time() - t0
    summary = {**{k: round(v, 2) for k, v in t.items()},
               "eval_engine": "hip"}
    with open(os.path.join(a.out, "run_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
