"""PESQ and STOI (reference ``F/audio/pesq.py``, ``F/audio/stoi.py``): thin wrappers over the ITU-T P.862 ``pesq``
and ``pystoi`` reference implementations, exactly like the reference.  Neither package is installed in this image, so
the metrics raise ``ModuleNotFoundError`` at construction / call time, as the reference does."""
from typing import Any

import numpy as np
import torch
from torch import Tensor

from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.imports import _PESQ_AVAILABLE, _PYSTOI_AVAILABLE


def perceptual_evaluation_speech_quality(preds: Tensor, target: Tensor, fs: int, mode: str,
                                         keep_same_device: bool = False, n_processes: int = 1) -> Tensor:
    """PESQ score per sample (``F/audio/pesq.py:24``)."""
    if not _PESQ_AVAILABLE:
        raise ModuleNotFoundError(
            "PESQ metric requires that pesq is installed. Either install as `pip install torchmetrics[audio]` or"
            " `pip install pesq`.")
    import pesq as pesq_backend

    if fs not in (8000, 16000):
        raise ValueError(f"Expected argument `fs` to either be 8000 or 16000 but got {fs}")
    if mode not in ("wb", "nb"):
        raise ValueError(f"Expected argument `mode` to either be 'wb' or 'nb' but got {mode}")
    _check_same_shape(preds, target)
    if preds.ndim == 1:
        val = torch.tensor(pesq_backend.pesq(fs, target.detach().cpu().numpy(), preds.detach().cpu().numpy(), mode))
    else:
        p = preds.reshape(-1, preds.shape[-1]).detach().cpu().numpy()
        t = target.reshape(-1, preds.shape[-1]).detach().cpu().numpy()
        if n_processes != 1:
            vals = pesq_backend.pesq_batch(fs, t, p, mode, n_processor=n_processes)
            vals = np.array(vals)
        else:
            vals = np.array([pesq_backend.pesq(fs, t[i], p[i], mode) for i in range(p.shape[0])])
        val = torch.from_numpy(vals).reshape(preds.shape[:-1])
    return val.to(preds.device) if keep_same_device else val


def short_time_objective_intelligibility(preds: Tensor, target: Tensor, fs: int, extended: bool = False,
                                         keep_same_device: bool = False) -> Tensor:
    """STOI / ESTOI per sample (``F/audio/stoi.py:25``)."""
    if not _PYSTOI_AVAILABLE:
        raise ModuleNotFoundError(
            "ShortTimeObjectiveIntelligibility metric requires that `pystoi` is installed."
            " Either install as `pip install torchmetrics[audio]` or `pip install pystoi`.")
    from pystoi import stoi as stoi_backend

    _check_same_shape(preds, target)
    if preds.ndim == 1:
        val = torch.tensor(stoi_backend(target.detach().cpu().numpy(), preds.detach().cpu().numpy(), fs, extended))
    else:
        p = preds.reshape(-1, preds.shape[-1]).detach().cpu().numpy()
        t = target.reshape(-1, preds.shape[-1]).detach().cpu().numpy()
        vals = np.array([stoi_backend(t[i], p[i], fs, extended) for i in range(p.shape[0])])
        val = torch.from_numpy(vals).reshape(preds.shape[:-1])
    return val.to(preds.device) if keep_same_device else val
