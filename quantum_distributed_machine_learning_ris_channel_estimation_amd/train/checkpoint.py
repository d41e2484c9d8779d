"""Reference-compatible checkpoint layout + atomic writes + resume files.

Layout (Runner_P128_QuantumNAT_onchipQNN.py:237-266, 416-426; Test.py:69-107):

  ./workspace/Pn_{P}/HDCE/
    Conv{s}_{bs}_{snr}dB_epoch{e}_DML.pth   {'conv':   state_dict with 'module.' prefix}
    Linear_{bs}_{snr}dB_epoch{e}_DML.pth    {'linear': state_dict with 'module.' prefix}
    Conv{s}_..._best_DML.pth / Linear_..._best_DML.pth        (best val NMSE)
    QSC_OPT_{bs}_{snr}dB_best_DML.pth / ..._epoch{e}_DML.pth  bare state_dict (no prefix)
    {bs}_{snr}dB_epoch{e}_DML_SC.pth        {'cnn': state_dict}     (name Test.py expects)
    QSC_optimized_best.pth                  {'model_state_dict': ...} (name Test.py expects)
    *_resume.pth                            optimizer state, epoch, best metric, RNG, LR
                                            (the reference cannot resume; these files never
                                             collide with the compatible names)

The ``module.`` prefix reproduces what a DataParallel-wrapped model saves (R:144-148).
Every file holds plain CPU tensors only, so ``torch.load(..., weights_only=True)``
works without this package.  Writes go to ``*.tmp`` then ``os.replace`` (atomic on
POSIX), on rank 0 only.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import numpy as np
import torch
import torch.nn as nn


def ckpt_dir(workspace: str, pilot_num: int, make: bool = True) -> str:
    d = os.path.join(workspace, f"Pn_{pilot_num}", "HDCE")
    if make:
        os.makedirs(d, exist_ok=True)
    return d


def plain_state_dict(module: nn.Module, prefix: str = "") -> Dict[str, torch.Tensor]:
    """CPU, contiguous, storage-owning copies (never the shared flat buffer)."""
    return {prefix + k: v.detach().to("cpu").clone().contiguous() for k, v in module.state_dict().items()}


def atomic_save(obj: Any, path: str) -> None:
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def hdce_names(bs: int, snr: int, tag: str):
    """tag = 'epoch{e}' or 'best'."""
    return ([f"Conv{s}_{bs}_{snr}dB_{tag}_DML.pth" for s in range(3)], f"Linear_{bs}_{snr}dB_{tag}_DML.pth")


def save_hdce(d: str, convs, fc: nn.Module, bs: int, snr: int, tag: str, dp_prefix: bool = True) -> None:
    pre = "module." if dp_prefix else ""
    conv_names, lin_name = hdce_names(bs, snr, tag)
    for name, m in zip(conv_names, convs):
        atomic_save({"conv": plain_state_dict(m, pre)}, os.path.join(d, name))
    atomic_save({"linear": plain_state_dict(fc, pre)}, os.path.join(d, lin_name))


def qsc_names(bs: int, snr: int, tag: str) -> str:
    return f"QSC_OPT_{bs}_{snr}dB_{tag}_DML.pth"


def save_qsc(d: str, model: nn.Module, bs: int, snr: int, tag: str, alias: bool = False) -> None:
    sd = plain_state_dict(model)
    atomic_save(sd, os.path.join(d, qsc_names(bs, snr, tag)))
    if alias:
        meta = {"n_qubits": model.num_qubits, "n_layers": model.n_layers, "n_classes": model.n_classes}
        atomic_save({"model_state_dict": sd, "qsc_config": meta}, os.path.join(d, "QSC_optimized_best.pth"))


def sc_name(bs: int, snr: int, tag: str) -> str:
    return f"{bs}_{snr}dB_{tag}_DML_SC.pth"


def save_sc(d: str, model: nn.Module, bs: int, snr: int, tag: str) -> None:
    atomic_save({"cnn": plain_state_dict(model, "module.")}, os.path.join(d, sc_name(bs, snr, tag)))


def load_model_state_dict(model: nn.Module, filepath: str, fallback_key: Optional[str] = None,
                          map_location="cpu", verbose: bool = True) -> None:
    """Test.py:23-62 semantics: pick ckpt[fallback_key] | ckpt['state_dict'] | ckpt, reconcile the
    DataParallel 'module.' prefix in either direction, strict load.  Safe loader only."""
    if not os.path.exists(filepath):
        raise FileNotFoundError(f"Model file not found: {filepath}")
    ckpt = torch.load(filepath, map_location=map_location, weights_only=True)
    if isinstance(ckpt, dict) and fallback_key and fallback_key in ckpt:
        sd = ckpt[fallback_key]
    elif isinstance(ckpt, dict) and "state_dict" in ckpt:
        sd = ckpt["state_dict"]
    else:
        sd = ckpt
    wrapped = hasattr(model, "module")
    first = next(iter(sd))
    if first.startswith("module.") and not wrapped:
        sd = {k[7:]: v for k, v in sd.items()}
    elif not first.startswith("module.") and wrapped:
        sd = {"module." + k: v for k, v in sd.items()}
    model.load_state_dict(sd)
    if verbose:
        print(f"Successfully loaded model from {filepath}")


def load_into(dst: torch.Tensor, src: torch.Tensor) -> None:
    with torch.no_grad():
        dst.copy_(src.to(dst.device, dst.dtype))


def rng_state() -> Dict[str, Any]:
    """RNG states as plain tensors (loadable with weights_only=True)."""
    st = {"torch": torch.get_rng_state(), "numpy": torch.from_numpy(np.random.get_state()[1].astype(np.int64))}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st: Dict[str, Any]) -> None:
    torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])


def save_resume(path: str, **state) -> None:
    atomic_save(state, path)


def load_resume(path: str) -> Optional[Dict[str, Any]]:
    if not os.path.exists(path):
        return None
    return torch.load(path, map_location="cpu", weights_only=True)
