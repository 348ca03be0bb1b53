"""Precision-recall curves and the shared curve machinery (binned HIP histogram + sort-based unbinned path).

Behavioural reference: ``F/classification/precision_recall_curve.py:28-1001``.  Differences in *how*:

* binned (``thresholds`` given): one pass of ``csrc/classification/curve.hip`` per update (LDS histogram over
  threshold buckets + suffix scan), no ``N x C x T`` temporary, no per-threshold loop and no host sync for the
  sigmoid/softmax decision (made on the device);
* unbinned (``thresholds=None``): the sigmoid/softmax decision is a device-side ``where`` (no sync); curves come from
  one sort per column.  AUROC / AP over many classes use the batched tie-aware formulas in
  :mod:`torchmetrics_amd.functional.classification.auroc` instead of a Python loop over classes.
"""
from typing import List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification import _sorted
from torchmetrics_amd.functional.classification.stat_scores import _check_flag, _Ctx
from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.compute import _safe_divide
from torchmetrics_amd.utilities.enums import ClassificationTask

Thresholds = Optional[Union[int, List[float], Tensor]]


# ------------------------------------------------------------------------------------------------ curve primitives
def _clf_curves(preds: Tensor, target: Tensor, tmode: int, pos_label: int = 1, ignore_index: Optional[int] = None,
                sample_weights: Optional[Tensor] = None):
    """``(fps_list, tps_list, thr_list, host_stats)`` for every column of ``preds`` from ONE sorted-curve launch."""
    out = _sorted.column_stats(preds, target, tmode, pos_label, ignore_index, ops.EMIT_CURVE, sample_weights)
    return _sorted.split_curves(out, preds.dtype)


def _clf_pr_curves(preds: Tensor, target: Tensor, tmode: int,
                   ignore_index: Optional[int] = None) -> Tuple[List[Tensor], List[Tensor], List[Tensor]]:
    """Every column's PR curve from one sorted-curve launch and one ``[S, N + 1]`` epilogue; the per-class tensors
    are views of it (``_sorted.pr_curves``)."""
    out = _sorted.column_stats(preds, target, tmode, 1, ignore_index, ops.EMIT_CURVE)
    return _sorted.pr_curves(out, preds.dtype)


def _binary_clf_curve(
    preds: Tensor,
    target: Tensor,
    sample_weights: Optional[Union[Sequence, Tensor]] = None,
    pos_label: int = 1,
) -> Tuple[Tensor, Tensor, Tensor]:
    """False/true positive counts at every distinct score (descending), as in sklearn's ``_binary_clf_curve``."""
    with torch.no_grad():
        if sample_weights is not None and not isinstance(sample_weights, Tensor):
            sample_weights = torch.tensor(sample_weights, device=preds.device, dtype=torch.float)
        if preds.ndim > target.ndim:
            preds = preds[:, 0]
        if preds.numel() == 0:
            e = torch.zeros(0, dtype=torch.float32, device=preds.device)
            return e, e.clone(), preds.reshape(-1)
        fps, tps, thr, _ = _clf_curves(preds.reshape(-1), target.reshape(-1), ops.CLF_T_BINARY, pos_label,
                                       sample_weights=sample_weights)
        return fps[0], tps[0], thr[0]


def _adjust_threshold_arg(thresholds: Thresholds = None, device: Optional[torch.device] = None) -> Optional[Tensor]:
    if isinstance(thresholds, int):
        return torch.linspace(0, 1, thresholds, device=device)
    if isinstance(thresholds, list):
        return torch.tensor(thresholds, device=device)
    return thresholds


class _CurveWorkspace:
    """Per-metric device scratch for the binned kernel: sorted thresholds + permutation, histogram, control word.

    The histogram and control word are returned to zero by the kernel's finalize pass, so one allocation serves
    every update of the metric.
    """

    __slots__ = ("key", "thr_sorted", "perm", "hist", "ctl", "err")

    def __init__(self) -> None:
        self.key = None

    def get(self, thresholds: Tensor, hcols: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
        dev = thresholds.device
        key = (dev, thresholds.data_ptr(), thresholds.numel(), thresholds._version, hcols)
        if self.key != key:
            thr = thresholds.detach().to(torch.float64)
            self.thr_sorted, self.perm = thr.sort(stable=True)
            self.thr_sorted = self.thr_sorted.contiguous()
            self.hist = torch.zeros((thresholds.numel() + 1) * hcols * 2, dtype=torch.int32, device=dev)
            self.ctl = torch.zeros(1, dtype=torch.int32, device=dev)
            self.key = key
        return self.thr_sorted, self.perm, self.hist, self.ctl


def _binned_update(
    preds: Tensor,
    target: Tensor,
    thresholds: Tensor,
    mode: int,
    ignore_index: Optional[int],
    micro: bool = False,
    state: Optional[Tensor] = None,
    err: Optional[Tensor] = None,
    workspace: Optional[_CurveWorkspace] = None,
) -> Tensor:
    """Accumulate the ``[T, H, 2, 2]`` (or ``[T, 2, 2]``) multi-threshold confusion matrix of one batch."""
    if mode == ops.CURVE_BINARY:
        p, t, hcols = preds.reshape(-1), target.reshape(-1), 1
    else:
        c = preds.shape[1]
        p = preds.movedim(1, -1).reshape(-1, c) if preds.ndim > 2 else preds
        t = target.movedim(1, -1).reshape(-1, c) if (mode == ops.CURVE_MULTILABEL and target.ndim > 2) else target
        if mode == ops.CURVE_MULTICLASS:
            t = t.reshape(-1)
        hcols = 1 if micro else c
    n_thr = thresholds.numel()
    if state is None:
        shape = (n_thr, 2, 2) if hcols == 1 and (mode == ops.CURVE_BINARY or micro) else (n_thr, hcols, 2, 2)
        state = torch.zeros(shape, dtype=torch.long, device=preds.device)
    ws = workspace if workspace is not None else _CurveWorkspace()
    thr_sorted, perm, hist, ctl = ws.get(thresholds.to(preds.device), hcols)
    if err is None:
        from torchmetrics_amd.functional.classification.stat_scores import _sink_flag

        err = _sink_flag(preds.device)
    ops.curve_update(p, t, thr_sorted, perm, hist, ctl, state, err, mode, ignore_index, micro)
    return state


def _pr_from_confmat(state: Tensor) -> Tuple[Tensor, Tensor]:
    tps, fps, fns = state[..., 1, 1], state[..., 0, 1], state[..., 1, 0]
    return _safe_divide(tps, tps + fps), _safe_divide(tps, tps + fns)


# ------------------------------------------------------------------------------------------------------- binary
def _binary_precision_recall_curve_arg_validation(thresholds: Thresholds = None, ignore_index: Optional[int] = None) -> None:
    if thresholds is not None and not isinstance(thresholds, (list, int, Tensor)):
        raise ValueError(
            "Expected argument `thresholds` to either be an integer, list of floats or"
            f" tensor of floats, but got {thresholds}"
        )
    if isinstance(thresholds, int) and thresholds < 2:
        raise ValueError(
            f"If argument `thresholds` is an integer, expected it to be larger than 1, but got {thresholds}"
        )
    if isinstance(thresholds, list) and not all(isinstance(t, float) and 0 <= t <= 1 for t in thresholds):
        raise ValueError(
            "If argument `thresholds` is a list, expected all elements to be floats in the [0,1] range,"
            f" but got {thresholds}"
        )
    if isinstance(thresholds, Tensor) and not thresholds.ndim == 1:
        raise ValueError("If argument `thresholds` is an tensor, expected the tensor to be 1d")
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")


def _binary_precision_recall_curve_tensor_validation(
    preds: Tensor, target: Tensor, ignore_index: Optional[int] = None, check_values: bool = True
) -> None:
    """Shape/dtype checks; with ``check_values`` also the (host-syncing) target value check.

    GPU binned updates pass ``check_values=False``: the kernel records invalid targets in the metric's device flag.
    """
    _check_same_shape(preds, target)
    if target.is_floating_point():
        raise ValueError(
            "Expected argument `target` to be an int or long tensor with ground truth labels"
            f" but got tensor with dtype {target.dtype}"
        )
    if not preds.is_floating_point():
        raise ValueError(
            "Expected argument `preds` to be an floating tensor with probability/logit scores,"
            f" but got tensor with dtype {preds.dtype}"
        )
    if not check_values:
        return
    unique_values = torch.unique(target)
    bad = (unique_values != 0) & (unique_values != 1)
    if ignore_index is not None:
        bad &= unique_values != ignore_index
    if torch.any(bad):
        raise RuntimeError(
            f"Detected the following values in `target`: {unique_values} but expected only"
            f" the following values {[0, 1] if ignore_index is None else [ignore_index]}."
        )


def _prob_or(preds: Tensor, transformed: Tensor, considered: Optional[Tensor] = None) -> Tensor:
    """``transformed`` if any considered score is outside [0, 1] (NaN counts as outside), else ``preds``.

    Device-side select: no host round trip (the reference branches on ``torch.all(...)`` in Python).
    """
    inside = (preds >= 0) & (preds <= 1)
    if considered is not None:
        inside = inside | ~considered
    return torch.where(inside.all(), preds, transformed)


def _binary_precision_recall_curve_format(
    preds: Tensor,
    target: Tensor,
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
) -> Tuple[Tensor, Tensor, Optional[Tensor]]:
    """Unbinned-path formatting: flatten, drop ignored, sigmoid if the scores are logits."""
    preds = preds.flatten()
    target = target.flatten()
    if ignore_index is not None:
        keep = target != ignore_index
        preds = preds[keep]
        target = target[keep]
    if preds.numel():
        preds = _prob_or(preds, preds.sigmoid())
    return preds, target, _adjust_threshold_arg(thresholds, preds.device)


def _binary_precision_recall_curve_update(
    preds: Tensor,
    target: Tensor,
    thresholds: Optional[Tensor],
    ignore_index: Optional[int] = None,
    state: Optional[Tensor] = None,
    err: Optional[Tensor] = None,
    workspace: Optional[_CurveWorkspace] = None,
) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    """Binned: raw ``preds``/``target`` -> ``[T, 2, 2]`` (kernel). Unbinned: formatted ``(preds, target)``."""
    if thresholds is None:
        p, t, _ = _binary_precision_recall_curve_format(preds, target, None, ignore_index)
        return p, t
    return _binned_update(preds, target, thresholds, ops.CURVE_BINARY, ignore_index, False, state, err, workspace)


def _binary_precision_recall_curve_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    thresholds: Optional[Tensor],
    pos_label: int = 1,
) -> Tuple[Tensor, Tensor, Tensor]:
    if isinstance(state, Tensor) and thresholds is not None:
        precision, recall = _pr_from_confmat(state)
        one = torch.ones(1, dtype=precision.dtype, device=precision.device)
        return torch.cat([precision, one]), torch.cat([recall, torch.zeros_like(one)]), thresholds
    fps, tps, thr = _binary_clf_curve(state[0], state[1], pos_label=pos_label)
    return _pr_from_clf(fps, tps, thr)


def _pr_from_clf(fps: Tensor, tps: Tensor, thr: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    precision = tps / (tps + fps)
    recall = tps / tps[-1]
    one = torch.ones(1, dtype=precision.dtype, device=precision.device)
    precision = torch.cat([precision.flip(0), one])
    recall = torch.cat([recall.flip(0), torch.zeros_like(one)])
    return precision, recall, thr.flip(0).detach().clone()


def _binary_curve_state(
    preds: Tensor, target: Tensor, thresholds: Thresholds, ignore_index: Optional[int], validate_args: bool
) -> Tuple[Union[Tensor, Tuple[Tensor, Tensor]], Optional[Tensor]]:
    """Shared functional front end: validation + state for one batch (binned confmat or formatted inputs)."""
    thr = _adjust_threshold_arg(thresholds, preds.device)
    binned_gpu = thr is not None and preds.is_cuda
    if validate_args:
        _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
        _binary_precision_recall_curve_tensor_validation(preds, target, ignore_index, check_values=not binned_gpu)
    err = torch.zeros(1, dtype=torch.int32, device=preds.device) if (validate_args and binned_gpu) else None
    state = _binary_precision_recall_curve_update(preds, target, thr, ignore_index, err=err)
    if err is not None:
        _check_flag(err, _Ctx(ignore_index=ignore_index, num_classes=2))
    return state, thr


def binary_precision_recall_curve(
    preds: Tensor,
    target: Tensor,
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor, Tensor]:
    """Precision-recall pairs at every threshold for binary tasks (reference ``F/.../precision_recall_curve.py:330``).

    Returns ``(precision, recall, thresholds)``; precision/recall have one more element than thresholds (the
    ``(1, 0)`` end point).
    """
    state, thr = _binary_curve_state(preds, target, thresholds, ignore_index, validate_args)
    return _binary_precision_recall_curve_compute(state, thr)


# --------------------------------------------------------------------------------------------------- multiclass
def _multiclass_precision_recall_curve_arg_validation(
    num_classes: int,
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    average: Optional[Literal["micro", "macro"]] = None,
) -> None:
    if not isinstance(num_classes, int) or num_classes < 2:
        raise ValueError(f"Expected argument `num_classes` to be an integer larger than 1, but got {num_classes}")
    if average not in (None, "micro", "macro"):
        raise ValueError(f"Expected argument `average` to be one of None, 'micro' or 'macro', but got {average}")
    _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)


def _multiclass_precision_recall_curve_tensor_validation(
    preds: Tensor, target: Tensor, num_classes: int, ignore_index: Optional[int] = None, check_values: bool = True
) -> None:
    if not preds.ndim == target.ndim + 1:
        raise ValueError(
            f"Expected `preds` to have one more dimension than `target` but got {preds.ndim} and {target.ndim}"
        )
    if target.is_floating_point():
        raise ValueError(
            f"Expected argument `target` to be an int or long tensor, but got tensor with dtype {target.dtype}"
        )
    if not preds.is_floating_point():
        raise ValueError(f"Expected `preds` to be a float tensor, but got {preds.dtype}")
    if preds.shape[1] != num_classes:
        raise ValueError(
            "Expected `preds.shape[1]` to be equal to the number of classes but"
            f" got {preds.shape[1]} and {num_classes}."
        )
    if preds.shape[0] != target.shape[0] or preds.shape[2:] != target.shape[1:]:
        raise ValueError(
            "Expected the shape of `preds` should be (N, C, ...) and the shape of `target` should be (N, ...)"
            f" but got {preds.shape} and {target.shape}"
        )
    if not check_values:
        return
    num_unique_values = len(torch.unique(target))
    limit = num_classes if ignore_index is None else num_classes + 1
    if num_unique_values > limit:
        raise RuntimeError(
            "Detected more unique values in `target` than `num_classes`. Expected only "
            f"{limit} but found {num_unique_values} in `target`."
        )


def _multiclass_precision_recall_curve_format(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    average: Optional[Literal["micro", "macro"]] = None,
) -> Tuple[Tensor, Tensor, Optional[Tensor]]:
    """Unbinned-path formatting: ``[N, C, ...] -> [M, C]``, drop ignored rows, softmax if logits, micro flatten."""
    preds = preds.movedim(1, -1).reshape(-1, num_classes)
    target = target.flatten()
    if ignore_index is not None:
        keep = target != ignore_index
        preds = preds[keep]
        target = target[keep]
    if preds.numel():
        preds = _prob_or(preds, preds.softmax(1))
    if average == "micro":
        preds = preds.flatten()
        target = torch.nn.functional.one_hot(target, num_classes=num_classes).flatten()
    return preds, target, _adjust_threshold_arg(thresholds, preds.device)


def _multiclass_precision_recall_curve_update(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    thresholds: Optional[Tensor],
    average: Optional[Literal["micro", "macro"]] = None,
    ignore_index: Optional[int] = None,
    state: Optional[Tensor] = None,
    err: Optional[Tensor] = None,
    workspace: Optional[_CurveWorkspace] = None,
) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    if thresholds is None:
        p, t, _ = _multiclass_precision_recall_curve_format(preds, target, num_classes, None, ignore_index, average)
        return p, t
    return _binned_update(
        preds, target, thresholds, ops.CURVE_MULTICLASS, ignore_index, average == "micro", state, err, workspace
    )


def _multiclass_precision_recall_curve_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    num_classes: int,
    thresholds: Optional[Tensor],
    average: Optional[Literal["micro", "macro"]] = None,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    if average == "micro":
        return _binary_precision_recall_curve_compute(state, thresholds)
    if isinstance(state, Tensor) and thresholds is not None:
        precision, recall = _pr_from_confmat(state)
        ones = torch.ones(1, num_classes, dtype=precision.dtype, device=precision.device)
        precision = torch.cat([precision, ones]).T
        recall = torch.cat([recall, torch.zeros_like(ones)]).T
        thres = thresholds
        tensor_state = True
    else:
        precision_list, recall_list, thres_list = _clf_pr_curves(state[0], state[1], ops.CLF_T_OVR)
        tensor_state = False
    if average == "macro":
        if tensor_state:
            return _macro_average_curve(precision, recall, thres.repeat(num_classes), descending=False)
        return _macro_average_curve(precision_list, recall_list, torch.cat(thres_list), descending=False)
    if tensor_state:
        return precision, recall, thres
    return precision_list, recall_list, thres_list


def _macro_average_curve(xs: Union[Tensor, List[Tensor]], ys: Union[Tensor, List[Tensor]], all_thresholds: Tensor,
                         descending: bool) -> Tuple[Tensor, Tensor, Tensor]:
    """``average="macro"`` of C per-class curves ``(xs[c], ys[c])`` (rows of a ``[C, U]`` tensor or a ragged list):
    the grid is every curve point's x, sorted; the value at each grid point is the mean over the classes of each curve's
    linear interpolation there (reference: a per-class ``interp`` loop, F/classification/roc.py:189-200,
    precision_recall_curve.py:566-580).  All C interpolations run as one ``ops.interp_mean`` launch."""
    if isinstance(xs, Tensor):
        flat_x, flat_y = xs.reshape(-1), ys.reshape(-1)
        lengths = torch.full((xs.shape[0],), xs.shape[1], dtype=torch.int64)
    else:
        flat_x, flat_y = torch.cat(xs), torch.cat(ys)
        lengths = torch.tensor([x.numel() for x in xs], dtype=torch.int64)
    offsets = torch.zeros(lengths.numel() + 1, dtype=torch.int64)
    torch.cumsum(lengths, 0, out=offsets[1:])
    grid = flat_x.sort().values
    mean_y = ops.interp_mean(grid, flat_x, flat_y.to(flat_x.dtype), offsets.to(flat_x.device))
    return grid, mean_y, all_thresholds.sort(descending=descending).values


def _multiclass_curve_state(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    thresholds: Thresholds,
    average: Optional[str],
    ignore_index: Optional[int],
    validate_args: bool,
    arg_validation=None,
) -> Tuple[Union[Tensor, Tuple[Tensor, Tensor]], Optional[Tensor]]:
    thr = _adjust_threshold_arg(thresholds, preds.device)
    binned_gpu = thr is not None and preds.is_cuda
    if validate_args:
        if arg_validation is not None:
            arg_validation()
        else:
            _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index, average)
        _multiclass_precision_recall_curve_tensor_validation(
            preds, target, num_classes, ignore_index, check_values=not binned_gpu
        )
    err = torch.zeros(1, dtype=torch.int32, device=preds.device) if (validate_args and binned_gpu) else None
    state = _multiclass_precision_recall_curve_update(
        preds, target, num_classes, thr, average, ignore_index, err=err
    )
    if err is not None:
        _check_flag(err, _Ctx(ignore_index=ignore_index, num_classes=num_classes))
    return state, thr


def multiclass_precision_recall_curve(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    thresholds: Thresholds = None,
    average: Optional[Literal["micro", "macro"]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    """One-vs-rest precision-recall curves (reference ``F/.../precision_recall_curve.py:529``)."""
    state, thr = _multiclass_curve_state(preds, target, num_classes, thresholds, average, ignore_index, validate_args)
    return _multiclass_precision_recall_curve_compute(state, num_classes, thr, average)


# --------------------------------------------------------------------------------------------------- multilabel
def _multilabel_precision_recall_curve_arg_validation(
    num_labels: int, thresholds: Thresholds = None, ignore_index: Optional[int] = None
) -> None:
    _multiclass_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)


def _multilabel_precision_recall_curve_tensor_validation(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int] = None, check_values: bool = True
) -> None:
    _binary_precision_recall_curve_tensor_validation(preds, target, ignore_index, check_values)
    if preds.shape[1] != num_labels:
        raise ValueError(
            "Expected both `target.shape[1]` and `preds.shape[1]` to be equal to the number of labels"
            f" but got {preds.shape[1]} and expected {num_labels}"
        )


def _multilabel_precision_recall_curve_format(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
) -> Tuple[Tensor, Tensor, Optional[Tensor]]:
    """Unbinned-path formatting: ``[N, L, ...] -> [M, L]``, sigmoid if logits (ignored entries kept, masked later)."""
    preds = preds.movedim(1, -1).reshape(-1, num_labels)
    target = target.movedim(1, -1).reshape(-1, num_labels)
    if preds.numel():
        preds = _prob_or(preds, preds.sigmoid())
    return preds, target, _adjust_threshold_arg(thresholds, preds.device)


def _multilabel_precision_recall_curve_update(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    thresholds: Optional[Tensor],
    ignore_index: Optional[int] = None,
    state: Optional[Tensor] = None,
    err: Optional[Tensor] = None,
    workspace: Optional[_CurveWorkspace] = None,
) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    if thresholds is None:
        p, t, _ = _multilabel_precision_recall_curve_format(preds, target, num_labels, None, ignore_index)
        return p, t
    return _binned_update(preds, target, thresholds, ops.CURVE_MULTILABEL, ignore_index, False, state, err, workspace)


def _multilabel_masked_column(state: Tuple[Tensor, Tensor], i: int, ignore_index: Optional[int]) -> Tuple[Tensor, Tensor]:
    preds, target = state[0][:, i], state[1][:, i]
    if ignore_index is not None:
        keep = target != ignore_index
        preds, target = preds[keep], target[keep]
    return preds, target


def _multilabel_precision_recall_curve_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    num_labels: int,
    thresholds: Optional[Tensor],
    ignore_index: Optional[int] = None,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    if isinstance(state, Tensor) and thresholds is not None:
        precision, recall = _pr_from_confmat(state)
        ones = torch.ones(1, num_labels, dtype=precision.dtype, device=precision.device)
        return torch.cat([precision, ones]).T, torch.cat([recall, torch.zeros_like(ones)]).T, thresholds
    return _clf_pr_curves(state[0], state[1], ops.CLF_T_ELEM, ignore_index)


def _multilabel_curve_state(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    thresholds: Thresholds,
    ignore_index: Optional[int],
    validate_args: bool,
    arg_validation=None,
) -> Tuple[Union[Tensor, Tuple[Tensor, Tensor]], Optional[Tensor]]:
    thr = _adjust_threshold_arg(thresholds, preds.device)
    binned_gpu = thr is not None and preds.is_cuda
    if validate_args:
        if arg_validation is not None:
            arg_validation()
        else:
            _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
        _multilabel_precision_recall_curve_tensor_validation(
            preds, target, num_labels, ignore_index, check_values=not binned_gpu
        )
    err = torch.zeros(1, dtype=torch.int32, device=preds.device) if (validate_args and binned_gpu) else None
    state = _multilabel_precision_recall_curve_update(preds, target, num_labels, thr, ignore_index, err=err)
    if err is not None:
        _check_flag(err, _Ctx(ignore_index=ignore_index, num_classes=2))
    return state, thr


def multilabel_precision_recall_curve(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    """Per-label precision-recall curves (reference ``F/.../precision_recall_curve.py:830``)."""
    state, thr = _multilabel_curve_state(preds, target, num_labels, thresholds, ignore_index, validate_args)
    return _multilabel_precision_recall_curve_compute(state, num_labels, thr, ignore_index)


def _task_dispatch(task, binary_fn, multiclass_fn, multilabel_fn, num_classes, num_labels):
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_fn()
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_fn()
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_fn()
    raise ValueError(f"Task {task} not supported.")


def precision_recall_curve(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    thresholds: Thresholds = None,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[Literal["micro", "macro"]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    """Task wrapper over the binary / multiclass / multilabel precision-recall curves."""
    return _task_dispatch(
        task,
        lambda: binary_precision_recall_curve(preds, target, thresholds, ignore_index, validate_args),
        lambda: multiclass_precision_recall_curve(
            preds, target, num_classes, thresholds, average, ignore_index, validate_args
        ),
        lambda: multilabel_precision_recall_curve(preds, target, num_labels, thresholds, ignore_index, validate_args),
        num_classes,
        num_labels,
    )
