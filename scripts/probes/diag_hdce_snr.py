#!/usr/bin/env python3
"""HDCE high-SNR saturation diagnostic (GPU).

The HDCE is trained at 10 dB (reference R:23) and tested at 5-15 dB.  Its gain over LS shrinks with
SNR; three candidate limits are separated here, each on a freshly trained model (oracle routing, so
the scenario classifier plays no part):

  bn      eval-mode BN running statistics (collected at 10 dB) vs statistics re-estimated on the test
          SNR's own inputs -> how much of the loss is the BN statistics' SNR shift
  label   training labels = the noisy LS estimate (reference) vs the perfect channel -> the
          label-noise limit of the regression on a finite training set
  data    20k vs 60k samples per stream -> the finite-sample (over-fitting) limit

Per variant: NMSE (dB) vs the perfect channel at SNR 5..15 dB, plus 20 / 30 dB (the model's floor).

    python scripts/probes/diag_hdce_snr.py --epochs 100 --out reports/r2_hdce_snr.jsonl
"""
import argparse
import json
import math
import os
import shutil
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--test-len", type=int, default=10000)
    ap.add_argument("--variants", default="base,perfect_label,data60k")
    ap.add_argument("--out", default="reports/r2_hdce_snr.jsonl")
    a = ap.parse_args()
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.data.channel import (generate_mixed,
                                                                                              pack_channel,
                                                                                              pack_pilots)
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.models.estimators import NMSELoss
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import estimate_routed
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.evaluate import (recalibrate_bn,
                                                                                               restore_bn)
    from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.runner import Y2HRunner
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    crit = NMSELoss()
    db = lambda v: round(10 * math.log10(v), 2)
    snrs = (5, 7, 9, 11, 13, 15, 20, 30)
    for var in a.variants.split(","):
        ws = f"/tmp/diag_snr_{var}"
        shutil.rmtree(ws, ignore_errors=True)
        t0 = time.time()
        r = Y2HRunner(n_epochs=a.epochs, data_len=60000 if var == "data60k" else 20000, workspace=ws)
        if var == "perfect_label":
            tr, va = r.device_stores()
            tr.Hlabel.copy_(tr.Hperf)
        m = r.train_Conv_Linear_of_HDCE()
        convs, fc = list(m.convs), m.fc
        for c in convs:
            c.eval()
        fc.eval()
        rec = {"variant": var, "epochs": a.epochs, "train_s": round(time.time() - t0, 1),
               "val_db_last": db(r.val_HDCE_nmse[-1]),
               "snr": list(snrs), "ls": [], "hdce": [], "hdce_bn_recal": []}
        for snr in snrs:
            Yp, HLS, H, ind = generate_mixed(a.test_len, float(snr), 128, -1, base_seed=0,
                                             split="test@60000", device=m.fc_w.device)
            perf = pack_channel(H)
            x = pack_pilots(Yp, 128)
            rec["ls"].append(db(float(crit(pack_channel(HLS), perf))))
            rec["hdce"].append(db(float(crit(estimate_routed(convs, fc, x, ind), perf))))
            saved = recalibrate_bn(convs, x, ind)
            rec["hdce_bn_recal"].append(db(float(crit(estimate_routed(convs, fc, x, ind), perf))))
            restore_bn(convs, saved)
        print(json.dumps(rec), flush=True)
        with open(a.out, "a") as f:
            f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
