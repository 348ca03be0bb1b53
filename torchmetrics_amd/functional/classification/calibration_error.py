"""Expected / max / RMS calibration error (reference ``F/classification/calibration_error.py:29-280``).

Binning is one ``bucketize`` + three ``scatter_add`` passes fused into a single ``index_add`` over a stacked
``[n, 3]`` source (count, confidence, accuracy), and the sigmoid/softmax decision is a device-side select.
"""
from typing import Optional, Tuple, Union

import torch
from torch import Tensor

from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification.precision_recall_curve import _prob_or
from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.enums import ClassificationTaskNoMultilabel
from torchmetrics_amd.utils.validation import TARGET_OUT_OF_RANGE as _TARGET_OUT_OF_RANGE


def _binning_bucketize(confidences: Tensor, accuracies: Tensor, bin_boundaries: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    if confidences.is_cuda and confidences.dtype == torch.float32 and len(bin_boundaries) <= 4096:
        # one pass with an LDS (count, Σconf, Σacc) histogram instead of bucketize + stack + index_add
        sums = ops.calibration_bins(confidences, accuracies.float(), bin_boundaries)
        count = sums[:, 0]
        return (torch.nan_to_num(sums[:, 2] / count), torch.nan_to_num(sums[:, 1] / count), count / count.sum())
    accuracies = accuracies.to(dtype=confidences.dtype)
    nb = len(bin_boundaries)
    idx = torch.bucketize(confidences, bin_boundaries, right=True) - 1
    src = torch.stack([torch.ones_like(confidences), confidences, accuracies], dim=1)
    sums = torch.zeros(nb, 3, dtype=confidences.dtype, device=confidences.device).index_add_(0, idx, src)
    count = sums[:, 0]
    conf_bin = torch.nan_to_num(sums[:, 1] / count)
    acc_bin = torch.nan_to_num(sums[:, 2] / count)
    prop_bin = count / count.sum()
    return acc_bin, conf_bin, prop_bin


_BOUNDARIES: dict = {}  # (n_bins, dtype, device) -> linspace(0, 1, n_bins + 1): one launch saved per compute()


def _ce_compute(
    confidences: Tensor,
    accuracies: Tensor,
    bin_boundaries: Union[Tensor, int],
    norm: str = "l1",
    debias: bool = False,
) -> Tensor:
    if isinstance(bin_boundaries, int):
        key = (bin_boundaries, confidences.dtype, confidences.device)
        cached = _BOUNDARIES.get(key)
        if cached is None:
            cached = _BOUNDARIES[key] = torch.linspace(0, 1, bin_boundaries + 1, dtype=confidences.dtype,
                                                       device=confidences.device)
        bin_boundaries = cached
    if norm not in {"l1", "l2", "max"}:
        raise ValueError(f"Argument `norm` is expected to be one of 'l1', 'l2', 'max' but got {norm}")
    if (norm != "l2" and confidences.is_cuda and confidences.dtype == torch.float32
            and len(bin_boundaries) <= 4096):
        with torch.no_grad():
            return ops.calibration_error_l1_max(confidences, accuracies.float(), bin_boundaries, norm)
    with torch.no_grad():
        acc_bin, conf_bin, prop_bin = _binning_bucketize(confidences, accuracies, bin_boundaries)
    if norm == "l1":
        return torch.sum(torch.abs(acc_bin - conf_bin) * prop_bin)
    if norm == "max":
        return torch.max(torch.abs(acc_bin - conf_bin))
    ce = torch.sum(torch.pow(acc_bin - conf_bin, 2) * prop_bin)
    if debias:
        debias_bins = (acc_bin * (acc_bin - 1) * prop_bin) / (prop_bin * accuracies.size()[0] - 1)
        ce += torch.sum(torch.nan_to_num(debias_bins))
    return torch.sqrt(ce) if ce > 0 else torch.tensor(0)


def _binary_calibration_error_arg_validation(
    n_bins: int, norm: Literal["l1", "l2", "max"] = "l1", ignore_index: Optional[int] = None
) -> None:
    if not isinstance(n_bins, int) or n_bins < 1:
        raise ValueError(f"Expected argument `n_bins` to be an integer larger than 0, but got {n_bins}")
    allowed_norm = ("l1", "l2", "max")
    if norm not in allowed_norm:
        raise ValueError(f"Expected argument `norm` to be one of {allowed_norm}, but got {norm}.")
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")


def _binary_float_preds_validation(preds: Tensor, target: Tensor, ignore_index: Optional[int]) -> None:
    """Binary target in {0, 1, ignore} and floating preds (the checks the reference runs before calibration/hinge)."""
    _check_same_shape(preds, target)
    if target.is_floating_point():
        raise ValueError(
            "Expected argument `target` to be an int or long tensor with ground truth labels"
            f" but got tensor with dtype {target.dtype}"
        )
    if not preds.is_floating_point():
        raise ValueError(
            "Expected argument `preds` to be floating tensor with probabilities/logits"
            f" but got tensor with dtype {preds.dtype}"
        )
    uniq = torch.unique(target)
    bad = (uniq != 0) & (uniq != 1)
    if ignore_index is not None:
        bad &= uniq != ignore_index
    if bad.any():
        raise RuntimeError(
            f"Detected the following values in `target`: {uniq} but expected only"
            f" the following values {[0, 1] if ignore_index is None else [0, 1, ignore_index]}."
        )


def _multiclass_float_preds_validation(preds: Tensor, target: Tensor, num_classes: int,
                                       ignore_index: Optional[int], flag: Optional[Tensor] = None,
                                       check_values: bool = True) -> None:
    """Shape / dtype checks on the host; the target range check is a device-side flag (raised at ``compute``)
    when a metric error word ``flag`` is given, else an immediate host check."""
    if preds.ndim != target.ndim + 1:
        raise ValueError("Expected `preds` to have one more dimension than `target`.")
    if not preds.is_floating_point():
        raise ValueError(
            "Expected argument `preds` to be floating tensor with probabilities/logits"
            f" but got tensor with dtype {preds.dtype}"
        )
    if target.is_floating_point():
        raise ValueError(f"Expected argument `target` to be an int or long tensor, but got {target.dtype}")
    if preds.shape[1] != num_classes:
        raise ValueError("If `preds` have one dimension more than `target`, `preds.shape[1]` should be"
                         " equal to number of classes.")
    if preds.shape[2:] != target.shape[1:]:
        raise ValueError("If `preds` have one dimension more than `target`, the shape of `preds` should be"
                         " (N, C, ...), and the shape of `target` should be (N, ...).")
    if not check_values:  # the caller's kernel raises the target range bit itself
        return
    bad = (target < 0) | (target >= num_classes)
    if ignore_index is not None:
        bad &= target != ignore_index
    if flag is not None:
        flag.bitwise_or_(bad.any().to(torch.int32) * _TARGET_OUT_OF_RANGE)
    elif bool(bad.any()):
        raise RuntimeError(f"Detected target values outside [0, {num_classes}).")


def _binary_format(preds: Tensor, target: Tensor, ignore_index: Optional[int]) -> Tuple[Tensor, Tensor]:
    """Flatten, drop ignored, sigmoid if logits (device-side decision)."""
    preds, target = preds.flatten(), target.flatten()
    if ignore_index is not None:
        keep = target != ignore_index
        preds, target = preds[keep], target[keep]
    if preds.is_floating_point() and preds.numel():
        preds = _prob_or(preds, preds.sigmoid())
    return preds, target


def _multiclass_format(preds: Tensor, target: Tensor, ignore_index: Optional[int]) -> Tuple[Tensor, Tensor]:
    """``[N, C, ...] -> [M, C]`` rows aligned with ``target.flatten()``, ignored rows dropped."""
    preds = preds.movedim(1, -1).reshape(-1, preds.shape[1])
    target = target.flatten()
    if ignore_index is not None:
        keep = target != ignore_index
        preds, target = preds[keep], target[keep]
    return preds, target


def _binary_calibration_error_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    return preds, target


def binary_calibration_error(
    preds: Tensor,
    target: Tensor,
    n_bins: int = 15,
    norm: Literal["l1", "l2", "max"] = "l1",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Top-label calibration error of binary probabilities (ECE for ``l1``, MCE for ``max``, RMSCE for ``l2``)."""
    if validate_args:
        _binary_calibration_error_arg_validation(n_bins, norm, ignore_index)
        _binary_float_preds_validation(preds, target, ignore_index)
    preds, target = _binary_format(preds, target, ignore_index)
    confidences, accuracies = _binary_calibration_error_update(preds, target)
    return _ce_compute(confidences, accuracies, n_bins, norm)


def _multiclass_calibration_error_arg_validation(
    num_classes: int, n_bins: int, norm: Literal["l1", "l2", "max"] = "l1", ignore_index: Optional[int] = None
) -> None:
    if not isinstance(num_classes, int) or num_classes < 2:
        raise ValueError(f"Expected argument `num_classes` to be an integer larger than 1, but got {num_classes}")
    _binary_calibration_error_arg_validation(n_bins, norm, ignore_index)


def _multiclass_calibration_error_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    if preds.numel():
        preds = _prob_or(preds, preds.softmax(1))
    confidences, predictions = preds.max(dim=1)
    accuracies = predictions.eq(target)
    return confidences.float(), accuracies.float()


def multiclass_calibration_error(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    n_bins: int = 15,
    norm: Literal["l1", "l2", "max"] = "l1",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Top-label calibration error for multiclass probabilities / logits."""
    if validate_args:
        _multiclass_calibration_error_arg_validation(num_classes, n_bins, norm, ignore_index)
        _multiclass_float_preds_validation(preds, target, num_classes, ignore_index)
    preds, target = _multiclass_format(preds, target, ignore_index)
    confidences, accuracies = _multiclass_calibration_error_update(preds, target)
    return _ce_compute(confidences, accuracies, n_bins, norm)


def calibration_error(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass"],
    n_bins: int = 15,
    norm: Literal["l1", "l2", "max"] = "l1",
    num_classes: Optional[int] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    task = ClassificationTaskNoMultilabel.from_str(task)
    if task == ClassificationTaskNoMultilabel.BINARY:
        return binary_calibration_error(preds, target, n_bins, norm, ignore_index, validate_args)
    if task == ClassificationTaskNoMultilabel.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_calibration_error(preds, target, num_classes, n_bins, norm, ignore_index, validate_args)
    raise ValueError(f"Expected argument `task` to either be `'binary'` or `'multiclass'` but got {task}")
