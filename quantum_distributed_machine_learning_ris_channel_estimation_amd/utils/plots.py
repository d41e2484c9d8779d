"""Plot helpers reproducing the reference's two published figures.

FIG1 ``channel estimation performace comparison.png`` (Test.py:277-319): NMSE (dB) vs SNR
for LS / MMSE / HDCE-classical / HDCE-quantum, and SC accuracy vs SNR.
FIG2 ``Loss Curve.png``: per-epoch training loss of the CNN and QML classifiers.
"""
from __future__ import annotations

from typing import Dict, Sequence


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def plot_fig1(res: Dict, path: str) -> None:
    plt = _plt()
    snr = res["SNR_dB"]
    plt.figure(figsize=(15, 6))
    plt.subplot(1, 2, 1)
    plt.plot(snr, res["NMSE_LS_dB"], "k--", linewidth=2, marker="o", markersize=8, label="LS Algorithm")
    plt.plot(snr, res["NMSE_MMSE_dB"], "r--", linewidth=2, marker="s", markersize=8, label="MMSE Algorithm")
    if "NMSE_LMMSE_dB" in res:
        plt.plot(snr, res["NMSE_LMMSE_dB"], "m:", linewidth=2, marker="x", markersize=8, label="LMMSE (Wiener)")
    plt.plot(snr, res["NMSE_HDCE_Classical_dB"], "b-", linewidth=3, marker="^", markersize=10,
             label="HDCE (Classical SC)")
    if any(v == v for v in res["NMSE_HDCE_Quantum_dB"]):
        plt.plot(snr, res["NMSE_HDCE_Quantum_dB"], "g-", linewidth=3, marker="d", markersize=10,
                 label="HDCE (Quantum SC)")
    plt.grid(True, alpha=0.3)
    plt.legend(fontsize=10)
    plt.xlabel("SNR (dB)")
    plt.ylabel("NMSE (dB)")
    plt.title("Channel Estimation Performance Comparison")
    plt.xticks(snr)
    plt.ylim(-20, 5)
    plt.subplot(1, 2, 2)
    plt.plot(snr, res["Accuracy_Classical"], "b-", linewidth=3, marker="^", markersize=10, label="Classical SC")
    if any(v == v for v in res["Accuracy_Quantum"]):
        plt.plot(snr, res["Accuracy_Quantum"], "g-", linewidth=3, marker="d", markersize=10, label="Quantum SC")
    plt.grid(True, alpha=0.3)
    plt.legend(fontsize=10)
    plt.xlabel("SNR (dB)")
    plt.ylabel("Accuracy")
    plt.title("Scenario Classification Accuracy Comparison")
    plt.xticks(snr)
    plt.ylim(0, 1)
    plt.tight_layout()
    plt.savefig(path, dpi=150, bbox_inches="tight")
    plt.close()


def plot_fig2(curves: Dict[str, Sequence[float]], path: str) -> None:
    """curves: label -> per-epoch loss (e.g. {'CNN': [...], 'QML 4 bits': [...]})."""
    plt = _plt()
    plt.figure(figsize=(10, 5))
    for label, ys in curves.items():
        plt.plot(range(len(ys)), ys, linewidth=2, label=label)
    plt.grid(True, alpha=0.3)
    plt.xlabel("Epoch")
    plt.ylabel("Training loss (NLL)")
    plt.title("Loss Curve")
    plt.legend()
    plt.tight_layout()
    plt.savefig(path, dpi=150)
    plt.close()
