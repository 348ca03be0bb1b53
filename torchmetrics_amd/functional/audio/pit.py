"""Permutation invariant training (reference ``F/audio/pit.py``).

Speaker-wise mode evaluates the ``spk x spk`` metric matrix with ONE batched ``metric_func`` call on
``[B * spk * spk, ...]`` views instead of ``spk^2`` calls, and solves the assignment on the device by scoring every
permutation with a gather (no host sync) up to ``_MAX_EXHAUSTIVE_SPK`` speakers; beyond that a batched Hungarian
solve runs on the device (one wave per batch item, ``ops.linear_sum_assignment``) -- scipy on the host only for CPU
tensors, like the reference.
"""
from itertools import permutations
from typing import Any, Callable, Dict, Literal, Tuple

import numpy as np
import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.utilities.imports import _SCIPY_AVAILABLE

_MAX_EXHAUSTIVE_SPK = 5
_ps_dict: Dict[str, Tensor] = {}


def _gen_permutations(spk_num: int, device: torch.device) -> Tensor:
    key = f"{spk_num}{device}"
    if key not in _ps_dict:
        _ps_dict[key] = torch.tensor(list(permutations(range(spk_num))), device=device)
    return _ps_dict[key]


def _find_best_perm_by_exhaustive_method(metric_mtx: Tensor, eval_func: Callable) -> Tuple[Tensor, Tensor]:
    b, spk = metric_mtx.shape[:2]
    ps = _gen_permutations(spk, metric_mtx.device)  # [P, spk]
    # metric of permutation p = mean_t metric_mtx[:, t, ps[p, t]]
    per = torch.gather(metric_mtx, 2, ps.T[None].expand(b, spk, ps.shape[0])).mean(dim=1)
    best_metric, best_idx = eval_func(per, dim=1)
    return best_metric, ps[best_idx.detach()]


def _find_best_perm_by_linear_sum_assignment(metric_mtx: Tensor, eval_func: Callable) -> Tuple[Tensor, Tensor]:
    if metric_mtx.is_cuda:
        # batched Hungarian solve on the device (csrc/audio/lsa.hip): no host round trip
        perm = ops.linear_sum_assignment(metric_mtx, maximize=eval_func == torch.max)
    else:
        from scipy.optimize import linear_sum_assignment

        mm = metric_mtx.detach().cpu()
        perm = torch.tensor(np.array([linear_sum_assignment(m, eval_func == torch.max)[1] for m in mm]))
        perm = perm.to(metric_mtx.device)
    return torch.gather(metric_mtx, 2, perm[:, :, None]).mean([-1, -2]), perm


def permutation_invariant_training(preds: Tensor, target: Tensor, metric_func: Callable,
                                   mode: Literal["speaker-wise", "permutation-wise"] = "speaker-wise",
                                   eval_func: Literal["max", "min"] = "max", **kwargs: Any) -> Tuple[Tensor, Tensor]:
    """Best metric over speaker permutations and the permutation achieving it (``F/audio/pit.py:87``)."""
    if preds.shape[0:2] != target.shape[0:2]:
        raise RuntimeError(
            "Predictions and targets are expected to have the same shape at the batch and speaker dimensions")
    if eval_func not in ["max", "min"]:
        raise ValueError(f'eval_func can only be "max" or "min" but got {eval_func}')
    if mode not in ["speaker-wise", "permutation-wise"]:
        raise ValueError(f'mode can only be "speaker-wise" or "permutation-wise" but got {eval_func}')
    if target.ndim < 2:
        raise ValueError(f"Inputs must be of shape [batch, spk, ...], got {target.shape} and {preds.shape} instead")
    eval_op = torch.max if eval_func == "max" else torch.min
    b, spk = target.shape[0:2]
    if mode == "permutation-wise":
        perms = _gen_permutations(spk, preds.device)
        n_perm = perms.shape[0]
        ppreds = torch.index_select(preds, 1, perms.reshape(-1)).reshape(b * n_perm, *preds.shape[1:])
        ptarget = target.repeat_interleave(n_perm, dim=0)
        m = metric_func(ppreds, ptarget, **kwargs)
        m = torch.mean(m.reshape(b, n_perm, -1), dim=-1)
        best_metric, best_idx = eval_op(m, dim=1)
        return best_metric, perms[best_idx.detach()]
    # all (target t, pred p) pairs in one call: rows ordered (batch, t, p)
    tail = preds.shape[2:]
    pp = preds[:, None].expand(b, spk, spk, *tail).reshape(b * spk * spk, *tail)
    tt = target[:, :, None].expand(b, spk, spk, *tail).reshape(b * spk * spk, *tail)
    metric_mtx = metric_func(pp, tt, **kwargs).reshape(b, spk, spk)
    if spk <= _MAX_EXHAUSTIVE_SPK or not (_SCIPY_AVAILABLE or metric_mtx.is_cuda):
        return _find_best_perm_by_exhaustive_method(metric_mtx, eval_op)
    return _find_best_perm_by_linear_sum_assignment(metric_mtx, eval_op)


def pit_permutate(preds: Tensor, perm: Tensor) -> Tensor:
    """Reorder the speaker axis of ``preds [B, spk, ...]`` by ``perm [B, spk]``."""
    idx = perm.reshape(*perm.shape, *([1] * (preds.ndim - 2))).expand_as(preds)
    return torch.gather(preds, 1, idx)
