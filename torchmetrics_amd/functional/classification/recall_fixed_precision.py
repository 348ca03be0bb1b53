"""Operating-point metrics read off the PR / ROC curves.

Recall @ fixed precision and precision @ fixed recall (reference ``F/classification/recall_fixed_precision.py``,
``precision_fixed_recall.py``), sensitivity @ specificity and specificity @ sensitivity (reference
``F/classification/sensitivity_specificity.py``, ``specificity_sensitivity.py`` incl. the deprecated misspelled
``specicity_at_sensitivity`` alias).  Curve states come from the shared binned HIP histogram / unbinned sort path.
"""
import inspect
import warnings
from typing import Callable, List, Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd.functional.classification.precision_recall_curve import (
    Thresholds,
    _binary_curve_state,
    _binary_precision_recall_curve_arg_validation,
    _binary_precision_recall_curve_compute,
    _multiclass_curve_state,
    _multiclass_precision_recall_curve_arg_validation,
    _multiclass_precision_recall_curve_compute,
    _multilabel_curve_state,
    _multilabel_precision_recall_curve_arg_validation,
    _multilabel_precision_recall_curve_compute,
    _task_dispatch,
)
from torchmetrics_amd.functional.classification.roc import (
    _binary_roc_compute,
    _multiclass_roc_compute,
    _multilabel_roc_compute,
)


# ------------------------------------------------------------------------------------------------ reductions
def _lexargmax(x: Tensor) -> Tensor:
    """Indices of the lexicographic maximum rows of ``x`` (column 0 first, ties broken by later columns)."""
    idx: Optional[Tensor] = None
    for k in range(x.shape[1]):
        col = x[idx, k] if idx is not None else x[:, k]
        z = torch.where(col == col.max())[0]
        idx = z if idx is None else idx[z]
        if len(idx) < 2:
            break
    if idx is None:
        raise ValueError("Failed to extract index")
    return idx


def _recall_at_precision(
    precision: Tensor, recall: Tensor, thresholds: Tensor, min_precision: float
) -> Tuple[Tensor, Tensor]:
    max_recall = torch.tensor(0.0, device=recall.device, dtype=recall.dtype)
    best_threshold = torch.tensor(0)
    n = min(t.shape[0] for t in (recall, precision, thresholds))
    zipped = torch.vstack((recall[:n], precision[:n], thresholds[:n].to(recall.dtype))).T
    masked = zipped[zipped[:, 1] >= min_precision]
    if masked.shape[0] > 0:
        idx = _lexargmax(masked)[0]
        max_recall, _, best_threshold = masked[idx]
    if max_recall == 0.0:
        best_threshold = torch.tensor(1e6, device=thresholds.device, dtype=thresholds.dtype)
    return max_recall, best_threshold


def _precision_at_recall(
    precision: Tensor, recall: Tensor, thresholds: Tensor, min_recall: float
) -> Tuple[Tensor, Tensor]:
    n = min(t.shape[0] for t in (recall, precision, thresholds))
    zipped = torch.vstack((precision[:n], recall[:n], thresholds[:n].to(precision.dtype))).T
    masked = zipped[zipped[:, 1] >= min_recall]
    if masked.shape[0] > 0:
        max_precision, _, best_threshold = masked[_lexargmax(masked)[0]]
    else:
        max_precision = torch.tensor(0.0, device=precision.device, dtype=precision.dtype)
        best_threshold = torch.tensor(0)
    if max_precision == 0.0:
        best_threshold = torch.tensor(1e6, device=thresholds.device, dtype=thresholds.dtype)
    return max_precision, best_threshold


def _best_under_constraint(value: Tensor, constraint: Tensor, thresholds: Tensor, min_constraint: float):
    keep = constraint >= min_constraint
    if not keep.any():
        return (torch.tensor(0.0, device=value.device, dtype=value.dtype),
                torch.tensor(1e6, device=thresholds.device, dtype=thresholds.dtype))
    value, thresholds = value[keep], thresholds[keep]
    idx = torch.argmax(value)
    return value[idx], thresholds[idx]


def _convert_fpr_to_specificity(fpr: Tensor) -> Tensor:
    return 1 - fpr


def _sensitivity_at_specificity(sensitivity: Tensor, specificity: Tensor, thresholds: Tensor, min_specificity: float):
    return _best_under_constraint(sensitivity, specificity, thresholds, min_specificity)


def _specificity_at_sensitivity(specificity: Tensor, sensitivity: Tensor, thresholds: Tensor, min_sensitivity: float):
    return _best_under_constraint(specificity, sensitivity, thresholds, min_sensitivity)


# ---------------------------------------------------------------------------------------------- validation
def _check_min(name: str, value: float) -> None:
    if not isinstance(value, float) and not (0 <= value <= 1):
        raise ValueError(f"Expected argument `{name}` to be an float in the [0,1] range, but got {value}")


def _binary_recall_at_fixed_precision_arg_validation(min_precision: float, thresholds: Thresholds = None,
                                                     ignore_index: Optional[int] = None) -> None:
    _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
    _check_min("min_precision", min_precision)


def _multiclass_recall_at_fixed_precision_arg_validation(num_classes: int, min_precision: float,
                                                         thresholds: Thresholds = None,
                                                         ignore_index: Optional[int] = None) -> None:
    _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index)
    _check_min("min_precision", min_precision)


def _multilabel_recall_at_fixed_precision_arg_validation(num_labels: int, min_precision: float,
                                                         thresholds: Thresholds = None,
                                                         ignore_index: Optional[int] = None) -> None:
    _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
    _check_min("min_precision", min_precision)


# ------------------------------------------------------------------------------------------ compute helpers
def _curve_for(kind: str, task: str, state, thresholds, num: int = 0, ignore_index: Optional[int] = None):
    """``(value_a, value_b, thresholds)`` curves: PR -> (precision, recall); ROC -> (sensitivity, specificity)."""
    if kind == "pr":
        if task == "binary":
            return _binary_precision_recall_curve_compute(state, thresholds)
        if task == "multiclass":
            return _multiclass_precision_recall_curve_compute(state, num, thresholds)
        return _multilabel_precision_recall_curve_compute(state, num, thresholds, ignore_index)
    if task == "binary":
        fpr, tpr, thr = _binary_roc_compute(state, thresholds)
        return tpr, _convert_fpr_to_specificity(fpr), thr
    if task == "multiclass":
        fpr, tpr, thr = _multiclass_roc_compute(state, num, thresholds)
    else:
        fpr, tpr, thr = _multilabel_roc_compute(state, num, thresholds, ignore_index)
    return tpr, [_convert_fpr_to_specificity(f) for f in fpr], thr


def _fixed_compute(kind: str, task: str, reduce_fn: Callable, state, thresholds, min_value: float, num: int = 0,
                   ignore_index: Optional[int] = None) -> Tuple[Tensor, Tensor]:
    a, b, thr = _curve_for(kind, task, state, thresholds, num, ignore_index)
    if task == "binary":
        return reduce_fn(a, b, thr, min_value)
    if isinstance(state, Tensor):
        res = [reduce_fn(x, y, thr, min_value) for x, y in zip(a, b)]
    else:
        res = [reduce_fn(x, y, t, min_value) for x, y, t in zip(a, b, thr)]
    return torch.stack([r[0] for r in res]), torch.stack([r[1] for r in res])


def _pr_reduce(kind: str) -> Callable:
    """Adapt the reductions to the curve tuple order produced by :func:`_curve_for`."""
    if kind == "recall@precision":
        return lambda p, r, t, m: _recall_at_precision(p, r, t, m)
    if kind == "precision@recall":
        return lambda p, r, t, m: _precision_at_recall(p, r, t, m)
    if kind == "sensitivity@specificity":
        return lambda sens, spec, t, m: _sensitivity_at_specificity(sens, spec, t, m)
    return lambda sens, spec, t, m: _specificity_at_sensitivity(spec, sens, t, m)


_KIND_CURVE = {
    "recall@precision": "pr",
    "precision@recall": "pr",
    "sensitivity@specificity": "roc",
    "specificity@sensitivity": "roc",
}


def _binary_fixed(kind, preds, target, min_value, thresholds, ignore_index, validate_args, min_name):
    if validate_args:
        _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
        _check_min(min_name, min_value)
    state, thr = _binary_curve_state(preds, target, thresholds, ignore_index, validate_args)
    return _fixed_compute(_KIND_CURVE[kind], "binary", _pr_reduce(kind), state, thr, min_value)


def _multiclass_fixed(kind, preds, target, num_classes, min_value, thresholds, ignore_index, validate_args, min_name):
    def arg_validation() -> None:
        _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index)
        _check_min(min_name, min_value)

    state, thr = _multiclass_curve_state(preds, target, num_classes, thresholds, None, ignore_index, validate_args,
                                         arg_validation=arg_validation)
    return _fixed_compute(_KIND_CURVE[kind], "multiclass", _pr_reduce(kind), state, thr, min_value, num_classes)


def _multilabel_fixed(kind, preds, target, num_labels, min_value, thresholds, ignore_index, validate_args, min_name):
    def arg_validation() -> None:
        _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
        _check_min(min_name, min_value)

    state, thr = _multilabel_curve_state(preds, target, num_labels, thresholds, ignore_index, validate_args,
                                         arg_validation=arg_validation)
    return _fixed_compute(_KIND_CURVE[kind], "multilabel", _pr_reduce(kind), state, thr, min_value, num_labels,
                          ignore_index)


# --------------------------------------------------------------------------------------- recall @ precision
def binary_recall_at_fixed_precision(preds: Tensor, target: Tensor, min_precision: float,
                                     thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                     validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    """Highest recall with precision >= ``min_precision`` and its threshold (binary)."""
    return _binary_fixed("recall@precision", preds, target, min_precision, thresholds, ignore_index, validate_args,
                         "min_precision")


def multiclass_recall_at_fixed_precision(preds: Tensor, target: Tensor, num_classes: int, min_precision: float,
                                         thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                         validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    """Per-class highest recall with precision >= ``min_precision`` and its threshold."""
    return _multiclass_fixed("recall@precision", preds, target, num_classes, min_precision, thresholds, ignore_index,
                             validate_args, "min_precision")


def multilabel_recall_at_fixed_precision(preds: Tensor, target: Tensor, num_labels: int, min_precision: float,
                                         thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                         validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    """Per-label highest recall with precision >= ``min_precision`` and its threshold."""
    return _multilabel_fixed("recall@precision", preds, target, num_labels, min_precision, thresholds, ignore_index,
                             validate_args, "min_precision")


def recall_at_fixed_precision(preds: Tensor, target: Tensor, task: Literal["binary", "multiclass", "multilabel"],
                              min_precision: float, thresholds: Thresholds = None, num_classes: Optional[int] = None,
                              num_labels: Optional[int] = None, ignore_index: Optional[int] = None,
                              validate_args: bool = True) -> Optional[Tuple[Tensor, Tensor]]:
    return _task_dispatch(
        task,
        lambda: binary_recall_at_fixed_precision(preds, target, min_precision, thresholds, ignore_index,
                                                 validate_args),
        lambda: multiclass_recall_at_fixed_precision(preds, target, num_classes, min_precision, thresholds,
                                                     ignore_index, validate_args),
        lambda: multilabel_recall_at_fixed_precision(preds, target, num_labels, min_precision, thresholds,
                                                     ignore_index, validate_args),
        num_classes, num_labels,
    )


# --------------------------------------------------------------------------------------- precision @ recall
def binary_precision_at_fixed_recall(preds: Tensor, target: Tensor, min_recall: float, thresholds: Thresholds = None,
                                     ignore_index: Optional[int] = None,
                                     validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    """Highest precision with recall >= ``min_recall`` and its threshold (binary)."""
    return _binary_fixed("precision@recall", preds, target, min_recall, thresholds, ignore_index, validate_args,
                         "min_precision")


def multiclass_precision_at_fixed_recall(preds: Tensor, target: Tensor, num_classes: int, min_recall: float,
                                         thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                         validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    return _multiclass_fixed("precision@recall", preds, target, num_classes, min_recall, thresholds, ignore_index,
                             validate_args, "min_precision")


def multilabel_precision_at_fixed_recall(preds: Tensor, target: Tensor, num_labels: int, min_recall: float,
                                         thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                         validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    return _multilabel_fixed("precision@recall", preds, target, num_labels, min_recall, thresholds, ignore_index,
                             validate_args, "min_precision")


def precision_at_fixed_recall(preds: Tensor, target: Tensor, task: Literal["binary", "multiclass", "multilabel"],
                              min_recall: float, thresholds: Thresholds = None, num_classes: Optional[int] = None,
                              num_labels: Optional[int] = None, ignore_index: Optional[int] = None,
                              validate_args: bool = True) -> Optional[Tuple[Tensor, Tensor]]:
    return _task_dispatch(
        task,
        lambda: binary_precision_at_fixed_recall(preds, target, min_recall, thresholds, ignore_index, validate_args),
        lambda: multiclass_precision_at_fixed_recall(preds, target, num_classes, min_recall, thresholds,
                                                     ignore_index, validate_args),
        lambda: multilabel_precision_at_fixed_recall(preds, target, num_labels, min_recall, thresholds,
                                                     ignore_index, validate_args),
        num_classes, num_labels,
    )


# --------------------------------------------------------------------------------- sensitivity @ specificity
def binary_sensitivity_at_specificity(preds: Tensor, target: Tensor, min_specificity: float,
                                      thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                      validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    """Highest sensitivity with specificity >= ``min_specificity`` and its threshold (binary)."""
    return _binary_fixed("sensitivity@specificity", preds, target, min_specificity, thresholds, ignore_index,
                         validate_args, "min_specificity")


def multiclass_sensitivity_at_specificity(preds: Tensor, target: Tensor, num_classes: int, min_specificity: float,
                                          thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                          validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    return _multiclass_fixed("sensitivity@specificity", preds, target, num_classes, min_specificity, thresholds,
                             ignore_index, validate_args, "min_specificity")


def multilabel_sensitivity_at_specificity(preds: Tensor, target: Tensor, num_labels: int, min_specificity: float,
                                          thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                          validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    return _multilabel_fixed("sensitivity@specificity", preds, target, num_labels, min_specificity, thresholds,
                             ignore_index, validate_args, "min_specificity")


def sensitivity_at_specificity(preds: Tensor, target: Tensor, task: Literal["binary", "multiclass", "multilabel"],
                               min_specificity: float, thresholds: Thresholds = None,
                               num_classes: Optional[int] = None, num_labels: Optional[int] = None,
                               ignore_index: Optional[int] = None, validate_args: bool = True):
    return _task_dispatch(
        task,
        lambda: binary_sensitivity_at_specificity(preds, target, min_specificity, thresholds, ignore_index,
                                                  validate_args),
        lambda: multiclass_sensitivity_at_specificity(preds, target, num_classes, min_specificity, thresholds,
                                                      ignore_index, validate_args),
        lambda: multilabel_sensitivity_at_specificity(preds, target, num_labels, min_specificity, thresholds,
                                                      ignore_index, validate_args),
        num_classes, num_labels,
    )


# --------------------------------------------------------------------------------- specificity @ sensitivity
def binary_specificity_at_sensitivity(preds: Tensor, target: Tensor, min_sensitivity: float,
                                      thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                      validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    """Highest specificity with sensitivity >= ``min_sensitivity`` and its threshold (binary)."""
    return _binary_fixed("specificity@sensitivity", preds, target, min_sensitivity, thresholds, ignore_index,
                         validate_args, "min_sensitivity")


def multiclass_specificity_at_sensitivity(preds: Tensor, target: Tensor, num_classes: int, min_sensitivity: float,
                                          thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                          validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    return _multiclass_fixed("specificity@sensitivity", preds, target, num_classes, min_sensitivity, thresholds,
                             ignore_index, validate_args, "min_sensitivity")


def multilabel_specificity_at_sensitivity(preds: Tensor, target: Tensor, num_labels: int, min_sensitivity: float,
                                          thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                                          validate_args: bool = True) -> Tuple[Tensor, Tensor]:
    return _multilabel_fixed("specificity@sensitivity", preds, target, num_labels, min_sensitivity, thresholds,
                             ignore_index, validate_args, "min_sensitivity")


def specificity_at_sensitivity(preds: Tensor, target: Tensor, task: Literal["binary", "multiclass", "multilabel"],
                               min_sensitivity: float, thresholds: Thresholds = None,
                               num_classes: Optional[int] = None, num_labels: Optional[int] = None,
                               ignore_index: Optional[int] = None, validate_args: bool = True):
    return _task_dispatch(
        task,
        lambda: binary_specificity_at_sensitivity(preds, target, min_sensitivity, thresholds, ignore_index,
                                                  validate_args),
        lambda: multiclass_specificity_at_sensitivity(preds, target, num_classes, min_sensitivity, thresholds,
                                                      ignore_index, validate_args),
        lambda: multilabel_specificity_at_sensitivity(preds, target, num_labels, min_sensitivity, thresholds,
                                                      ignore_index, validate_args),
        num_classes, num_labels,
    )


def specicity_at_sensitivity(*args, **kwargs):
    """Deprecated misspelled alias of :func:`specificity_at_sensitivity` (kept for API parity)."""
    warnings.warn(
        "This method has will be removed in 2.0.0. Use `specificity_at_sensitivity` instead.",
        DeprecationWarning,
        stacklevel=1,
    )
    return specificity_at_sensitivity(*args, **kwargs)


specicity_at_sensitivity.__signature__ = inspect.signature(specificity_at_sensitivity)  # type: ignore[attr-defined]
