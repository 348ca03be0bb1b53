"""Tensor/collection helpers (parity: reference ``S/utilities/data.py:25-245``).

Differences from the reference, by design:

* ``apply_to_collection`` is implemented here (no lightning-utilities dependency).
* ``_bincount`` never falls back to the O(N*C) one-hot mesh under deterministic mode: on ROCm the integer
  histogram is produced by our own HIP kernel whose integer atomics are order-independent, hence deterministic
  (reference fallback: ``S/utilities/data.py:203-205``).
"""
from typing import Any, Callable, Dict, List, Mapping, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor

METRIC_EPS = 1e-6


def apply_to_collection(
    data: Any,
    dtype: Union[type, Tuple[type, ...]],
    function: Callable,
    *args: Any,
    wrong_dtype: Optional[Union[type, Tuple[type, ...]]] = None,
    **kwargs: Any,
) -> Any:
    """Recursively apply ``function`` to every element of ``data`` that is an instance of ``dtype``."""
    if isinstance(data, dtype) and (wrong_dtype is None or not isinstance(data, wrong_dtype)):
        return function(data, *args, **kwargs)
    if getattr(data, "_tm_flat_mapping", False):
        # a mapping backed by one flat tensor (e.g. mAP's extended-summary IoU table): apply to the storage once
        return data.apply_flat(lambda t: apply_to_collection(t, dtype, function, *args, wrong_dtype=wrong_dtype,
                                                             **kwargs))
    if isinstance(data, Mapping):
        return type(data)(
            {k: apply_to_collection(v, dtype, function, *args, wrong_dtype=wrong_dtype, **kwargs) for k, v in data.items()}
        ) if not hasattr(data, "default_factory") else {
            k: apply_to_collection(v, dtype, function, *args, wrong_dtype=wrong_dtype, **kwargs) for k, v in data.items()
        }
    if isinstance(data, tuple) and hasattr(data, "_fields"):  # namedtuple
        return type(data)(*(apply_to_collection(d, dtype, function, *args, wrong_dtype=wrong_dtype, **kwargs) for d in data))
    if isinstance(data, (list, tuple)):
        return type(data)(apply_to_collection(d, dtype, function, *args, wrong_dtype=wrong_dtype, **kwargs) for d in data)
    return data


def dim_zero_cat(x: Union[Tensor, List[Tensor]]) -> Tensor:
    """Concatenate a list state along dim 0 (0-d elements are promoted to 1-d)."""
    if isinstance(x, Tensor):
        return x
    parts = [y.unsqueeze(0) if y.numel() == 1 and y.ndim == 0 else y for y in x]
    if not parts:
        raise ValueError("No samples to concatenate")
    return torch.cat(parts, dim=0)


def dim_zero_sum(x: Tensor) -> Tensor:
    return torch.sum(x, dim=0)


def dim_zero_mean(x: Tensor) -> Tensor:
    return torch.mean(x, dim=0)


def dim_zero_max(x: Tensor) -> Tensor:
    return torch.max(x, dim=0).values


def dim_zero_min(x: Tensor) -> Tensor:
    return torch.min(x, dim=0).values


def _flatten(x: Sequence) -> list:
    return [item for sub in x for item in sub]


def _flatten_dict(x: Dict) -> Tuple[Dict, bool]:
    """Flatten one level of nested dicts; returns the flat dict and whether a key collided."""
    out: Dict = {}
    dup = False
    for key, value in x.items():
        if isinstance(value, dict):
            for k, v in value.items():
                if k in out:
                    dup = True
                out[k] = v
        else:
            if key in out:
                dup = True
            out[key] = value
    return out, dup


def to_onehot(label_tensor: Tensor, num_classes: Optional[int] = None) -> Tensor:
    """``[N, d1, ...]`` integer labels -> ``[N, C, d1, ...]`` one-hot."""
    if num_classes is None:
        num_classes = int(label_tensor.max().detach().item() + 1)
    shape = (label_tensor.shape[0], num_classes, *label_tensor.shape[1:])
    out = torch.zeros(shape, dtype=label_tensor.dtype, device=label_tensor.device)
    return out.scatter_(1, label_tensor.long().unsqueeze(1).expand_as(out[:, :1]), 1.0)


def _top_k_with_half_precision_support(x: Tensor, k: int = 1, dim: int = 1) -> Tensor:
    if x.dtype == torch.half and not x.is_cuda:
        return torch.topk(x.float(), k=k, dim=dim).indices
    return torch.topk(x, k=k, dim=dim).indices


def select_topk(prob_tensor: Tensor, topk: int = 1, dim: int = 1) -> Tensor:
    """Binary int mask with a 1 at the ``topk`` largest entries along ``dim``."""
    out = torch.zeros_like(prob_tensor, dtype=torch.int32)
    if topk == 1:
        idx = prob_tensor.argmax(dim=dim, keepdim=True)
    else:
        idx = _top_k_with_half_precision_support(prob_tensor, k=topk, dim=dim)
    return out.scatter_(dim, idx, 1)


def to_categorical(x: Tensor, argmax_dim: int = 1) -> Tensor:
    return torch.argmax(x, dim=argmax_dim)


def _squeeze_scalar_element_tensor(x: Tensor) -> Tensor:
    return x.squeeze() if x.numel() == 1 else x


def _squeeze_if_scalar(data: Any) -> Any:
    return apply_to_collection(data, Tensor, _squeeze_scalar_element_tensor)


def _bincount(x: Tensor, minlength: Optional[int] = None) -> Tensor:
    """Deterministic integer histogram.

    CUDA (ROCm) tensors go through the HIP histogram kernel (``csrc/common/histogram.hip``); CPU uses ATen.
    """
    if minlength is None:
        minlength = int(x.max().item()) + 1 if x.numel() else 0
    if x.is_cuda:
        from torchmetrics_amd.ops import histogram

        return histogram(x, minlength)
    return torch.bincount(x, minlength=minlength)


def _cumsum(x: Tensor, dim: Optional[int] = 0, dtype: Optional[torch.dtype] = None) -> Tensor:
    return torch.cumsum(x, dim=dim, dtype=dtype)


def _flexible_bincount(x: Tensor) -> Tensor:
    """Counts of each unique value of ``x`` (values need not be contiguous)."""
    x = x - x.min()
    return torch.unique(x, return_counts=True)[1] if x.numel() else x.new_zeros(0)


def allclose(tensor1: Tensor, tensor2: Tensor) -> bool:
    if tensor1.dtype != tensor2.dtype:
        tensor2 = tensor2.to(dtype=tensor1.dtype)
    return torch.allclose(tensor1, tensor2)


__all__ = [
    "METRIC_EPS",
    "apply_to_collection",
    "dim_zero_cat",
    "dim_zero_sum",
    "dim_zero_mean",
    "dim_zero_max",
    "dim_zero_min",
    "to_onehot",
    "select_topk",
    "to_categorical",
]
