"""PESQ (reference ``F/audio/pesq.py``): a thin wrapper over the ITU-T P.862 ``pesq`` C implementation, exactly like
the reference (a host-side, standard-defined DSP pipeline; not a GPU target).  The package is not installed in this
image, so the metric raises ``ModuleNotFoundError`` at construction / call time, as the reference does.  STOI is
native: :mod:`torchmetrics_amd.functional.audio.stoi`."""
from typing import Any

import numpy as np
import torch
from torch import Tensor

from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.imports import _PESQ_AVAILABLE


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
