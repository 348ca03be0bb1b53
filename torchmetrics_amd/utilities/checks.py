"""Input checks (parity: reference ``S/utilities/checks.py``).

Value checks that would need a device->host sync on GPU tensors are NOT done here for CUDA inputs on the hot path;
those are folded into the HIP kernels as device-side error flags (see :mod:`torchmetrics_amd.utils.validation`).
The helpers below are shape/dtype checks (host metadata only) plus the retrieval checks and the developer tool
``check_forward_full_state_property`` (reference ``checks.py:636-738``).
"""
import inspect
from time import perf_counter
from typing import Any, Callable, Dict, Mapping, Optional, Sequence, Tuple

import torch
from torch import Tensor


def _check_for_empty_tensors(preds: Tensor, target: Tensor) -> bool:
    return preds.numel() == target.numel() == 0


def _check_same_shape(preds: Tensor, target: Tensor) -> None:
    if preds.shape != target.shape:
        raise RuntimeError(
            f"Predictions and targets are expected to have the same shape, but got {preds.shape} and {target.shape}."
        )


def _check_retrieval_target_and_prediction_types(
    preds: Tensor, target: Tensor, allow_non_binary_target: bool = False
) -> Tuple[Tensor, Tensor]:
    if target.dtype not in (torch.bool, torch.long, torch.int) and not torch.is_floating_point(target):
        raise ValueError("`target` must be a tensor of booleans, integers or floats")
    if not preds.is_floating_point():
        raise ValueError("`preds` must be a tensor of floats")
    if not allow_non_binary_target and (target.max() > 1 or target.min() < 0):
        raise ValueError("`target` must contain `binary` values")
    target = target.float() if target.is_floating_point() else target.long()
    return preds.float().flatten(), target.flatten()


def _check_retrieval_functional_inputs(
    preds: Tensor, target: Tensor, allow_non_binary_target: bool = False
) -> Tuple[Tensor, Tensor]:
    if preds.shape != target.shape:
        raise ValueError("`preds` and `target` must be of the same shape")
    if not preds.numel() or not preds.size():
        raise ValueError("`preds` and `target` must be non-empty and non-scalar tensors")
    return _check_retrieval_target_and_prediction_types(preds, target, allow_non_binary_target)


def _check_retrieval_inputs(
    indexes: Tensor,
    preds: Tensor,
    target: Tensor,
    allow_non_binary_target: bool = False,
    ignore_index: Optional[int] = None,
) -> Tuple[Tensor, Tensor, Tensor]:
    if indexes.shape != preds.shape or preds.shape != target.shape:
        raise ValueError("`indexes`, `preds` and `target` must be of the same shape")
    if indexes.dtype is not torch.long:
        raise ValueError("`indexes` must be a tensor of long integers")
    if ignore_index is not None:
        keep = target != ignore_index
        indexes, preds, target = indexes[keep], preds[keep], target[keep]
    if not indexes.numel() or not indexes.size():
        raise ValueError("`indexes`, `preds` and `target` must be non-empty and non-scalar tensors")
    preds, target = _check_retrieval_target_and_prediction_types(preds, target, allow_non_binary_target)
    return indexes.long().flatten(), preds, target


def _allclose_recursive(res1: Any, res2: Any, atol: float = 1e-6) -> bool:
    if isinstance(res1, Tensor):
        return torch.allclose(res1, res2, atol=atol)
    if isinstance(res1, str):
        return res1 == res2
    if isinstance(res1, Sequence):
        return all(_allclose_recursive(a, b) for a, b in zip(res1, res2))
    if isinstance(res1, Mapping):
        return all(_allclose_recursive(res1[k], res2[k]) for k in res1)
    return res1 == res2


def check_forward_full_state_property(
    metric_class: Any,
    init_args: Optional[Dict[str, Any]] = None,
    input_args: Optional[Dict[str, Any]] = None,
    num_update_to_compare: Sequence[int] = (10, 100, 1000),
    reps: int = 5,
) -> None:
    """Check whether ``full_state_update=False`` gives the same ``forward`` results, and whether it is faster.

    Prints a recommendation, like the reference developer tool.
    """
    init_args = init_args or {}
    input_args = input_args or {}

    class _Full(metric_class):  # type: ignore[misc,valid-type]
        full_state_update = True

    class _Part(metric_class):  # type: ignore[misc,valid-type]
        full_state_update = False

    full, part = _Full(**init_args), _Part(**init_args)
    equal = True
    try:  # a failure usually means the update needs the full state
        for _ in range(num_update_to_compare[0]):
            equal &= _allclose_recursive(full(**input_args), part(**input_args))
        equal &= _allclose_recursive(full.compute(), part.compute())
    except RuntimeError:
        equal = False
    if not equal:  # no timing needed: only the full-state mode is correct
        print("Recommended setting `full_state_update=True`")
        return
    res = torch.zeros(2, len(num_update_to_compare), reps)
    for i, metric in enumerate([full, part]):
        for j, steps in enumerate(num_update_to_compare):
            for r in range(reps):
                start = perf_counter()
                for _ in range(steps):
                    _ = metric(**input_args)
                end = perf_counter()
                res[i, j, r] = end - start
                metric.reset()
    mean = res.mean(-1)
    std = res.std(-1)
    for t, steps in enumerate(num_update_to_compare):
        print(f"Full state for {steps} steps took: {mean[0, t]:0.3f}+-{std[0, t]:0.3f}")
        print(f"Partial state for {steps} steps took: {mean[1, t]:0.3f}+-{std[1, t]:0.3f}")
    faster = bool(mean[1, -1] < mean[0, -1])
    print(f"Recommended setting `full_state_update={not faster}`")


def is_overridden(method_name: str, instance: object, parent: object) -> bool:
    """True if ``instance``'s class overrides ``parent.method_name``."""
    inst_attr = getattr(instance, method_name, None)
    if inst_attr is None:
        return False
    if hasattr(inst_attr, "__wrapped__"):
        inst_attr = inst_attr.__wrapped__
    if isinstance(inst_attr, Callable) and hasattr(inst_attr, "__code__") is False and hasattr(inst_attr, "__func__"):
        inst_attr = inst_attr.__func__
    parent_attr = getattr(parent, method_name, None)
    if parent_attr is None:
        raise ValueError("The parent should define the method")
    code_i = getattr(inst_attr, "__code__", None)
    code_p = getattr(parent_attr, "__code__", None)
    return code_i is not code_p


def _signature_params(fn: Callable) -> Dict[str, inspect.Parameter]:
    return dict(inspect.signature(fn).parameters)
