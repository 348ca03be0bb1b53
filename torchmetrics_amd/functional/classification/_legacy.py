"""Legacy (pre-0.11, task-less) classification input handling, still used by ``Dice``.

Behavioural reference: input-type inference and formatting ``S/utilities/checks.py`` (``_check_classification_inputs``,
``_input_format_classification``) and the legacy ``_stat_scores_update`` / ``_reduce_stat_scores``
(``F/classification/stat_scores.py:820-1080``).  Inputs are converted to a one-hot ``[N, C]`` / ``[N, C, X]``
layout; the tp/fp/tn/fn reductions are plain device tensor ops.
"""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_amd.utilities.data import select_topk, to_onehot
from torchmetrics_amd.utilities.enums import AverageMethod, DataType, MDMCAverageMethod


def _input_squeeze(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    if preds.shape[0] == 1:
        return preds.squeeze().unsqueeze(0), target.squeeze().unsqueeze(0)
    return preds.squeeze(), target.squeeze()


def _empty(preds: Tensor, target: Tensor) -> bool:
    return preds.numel() == target.numel() == 0


def _infer_case(preds: Tensor, target: Tensor) -> Tuple[DataType, int]:
    is_float = preds.is_floating_point()
    if preds.ndim == target.ndim:
        if preds.shape != target.shape:
            raise ValueError(
                "The `preds` and `target` should have the same shape,",
                f" got `preds` with shape={preds.shape} and `target` with shape={target.shape}.",
            )
        if is_float and target.numel() > 0 and target.max() > 1:
            raise ValueError(
                "If `preds` and `target` are of shape (N, ...) and `preds` are floats, `target` should be binary."
            )
        if preds.ndim == 1:
            case = DataType.BINARY if is_float else DataType.MULTICLASS
        else:
            case = DataType.MULTILABEL if is_float else DataType.MULTIDIM_MULTICLASS
        return case, (preds[0].numel() if preds.numel() > 0 else 0)
    if preds.ndim == target.ndim + 1:
        if not is_float:
            raise ValueError("If `preds` have one dimension more than `target`, `preds` should be a float tensor.")
        if preds.shape[2:] != target.shape[1:]:
            raise ValueError(
                "If `preds` have one dimension more than `target`, the shape of `preds` should be"
                " (N, C, ...), and the shape of `target` should be (N, ...)."
            )
        return (DataType.MULTICLASS if preds.ndim == 2 else DataType.MULTIDIM_MULTICLASS), (
            preds.shape[1] if preds.numel() > 0 else 0
        )
    raise ValueError(
        "Either `preds` and `target` both should have the (same) shape (N, ...), or `target` should be (N, ...)"
        " and `preds` should be (N, C, ...)."
    )


def _check_classification_inputs(
    preds: Tensor,
    target: Tensor,
    threshold: float,
    num_classes: Optional[int],
    multiclass: Optional[bool],
    top_k: Optional[int],
    ignore_index: Optional[int] = None,
) -> DataType:
    if not _empty(preds, target):
        if target.is_floating_point():
            raise ValueError("The `target` has to be an integer tensor.")
        if (ignore_index is None and target.min() < 0) or (ignore_index and ignore_index >= 0 and target.min() < 0):
            raise ValueError("The `target` has to be a non-negative tensor.")
        if not preds.is_floating_point() and preds.min() < 0:
            raise ValueError("If `preds` are integers, they have to be non-negative.")
        if preds.shape[0] != target.shape[0]:
            raise ValueError("The `preds` and `target` should have the same first dimension.")
        if multiclass is False and target.max() > 1:
            raise ValueError("If you set `multiclass=False`, then `target` should not exceed 1.")
        if multiclass is False and not preds.is_floating_point() and preds.max() > 1:
            raise ValueError("If you set `multiclass=False` and `preds` are integers, then `preds` should not exceed 1.")
    case, implied = _infer_case(preds, target)
    if preds.shape != target.shape:
        if multiclass is False and implied != 2:
            raise ValueError(
                "You have set `multiclass=False`, but have more than 2 classes in your data,"
                " based on the C dimension of `preds`."
            )
        if target.max() >= implied:
            raise ValueError(
                "The highest label in `target` should be smaller than the size of the `C` dimension of `preds`."
            )
    if num_classes:
        if case == DataType.BINARY:
            if num_classes > 2:
                raise ValueError("Your data is binary, but `num_classes` is larger than 2.")
            if num_classes == 2 and not multiclass:
                raise ValueError(
                    "Your data is binary and `num_classes=2`, but `multiclass` is not True."
                    " Set it to True if you want to transform binary data to multi-class format."
                )
            if num_classes == 1 and multiclass:
                raise ValueError(
                    "You have binary data and have set `multiclass=True`, but `num_classes` is 1."
                    " Either set `multiclass=None`(default) or set `num_classes=2`"
                    " to transform binary data to multi-class format."
                )
        elif case in (DataType.MULTICLASS, DataType.MULTIDIM_MULTICLASS):
            if num_classes == 1 and multiclass is not False:
                raise ValueError(
                    "You have set `num_classes=1`, but predictions are integers."
                    " If you want to convert (multi-dimensional) multi-class data with 2 classes"
                    " to binary/multi-label, set `multiclass=False`."
                )
            if num_classes > 1:
                if multiclass is False and implied != num_classes:
                    raise ValueError(
                        "You have set `multiclass=False`, but the implied number of classes "
                        " (from shape of inputs) does not match `num_classes`."
                    )
                if target.numel() > 0 and num_classes <= target.max():
                    raise ValueError("The highest label in `target` should be smaller than `num_classes`.")
                if preds.shape != target.shape and num_classes != implied:
                    raise ValueError("The size of C dimension of `preds` does not match `num_classes`.")
        else:
            if multiclass and num_classes != 2:
                raise ValueError(
                    "Your have set `multiclass=True`, but `num_classes` is not equal to 2."
                    " If you are trying to transform multi-label data to 2 class multi-dimensional"
                    " multi-class, you should set `num_classes` to either 2 or None."
                )
            if not multiclass and num_classes != implied:
                raise ValueError("The implied number of classes (from shape of inputs) does not match num_classes.")
    if top_k is not None:
        if case == DataType.BINARY:
            raise ValueError("You can not use `top_k` parameter with binary data.")
        if not isinstance(top_k, int) or top_k <= 0:
            raise ValueError("The `top_k` has to be an integer larger than 0.")
        if not preds.is_floating_point():
            raise ValueError("You have set `top_k`, but you do not have probability predictions.")
        if multiclass is False:
            raise ValueError("If you set `multiclass=False`, you can not set `top_k`.")
        if case == DataType.MULTILABEL and multiclass:
            raise ValueError(
                "If you want to transform multi-label data to 2 class multi-dimensional"
                "multi-class data using `multiclass=True`, you can not use `top_k`."
            )
        if top_k >= implied:
            raise ValueError("The `top_k` has to be strictly smaller than the `C` dimension of `preds`.")
    return case


def _input_format_classification(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    top_k: Optional[int] = None,
    num_classes: Optional[int] = None,
    multiclass: Optional[bool] = None,
    ignore_index: Optional[int] = None,
) -> Tuple[Tensor, Tensor, DataType]:
    """Infer the input case and convert to binary one-hot ``[N, C]`` / ``[N, C, X]`` int tensors."""
    preds, target = _input_squeeze(preds, target)
    if preds.dtype == torch.float16:
        preds = preds.float()
    case = _check_classification_inputs(preds, target, threshold, num_classes, multiclass, top_k, ignore_index)
    if case in (DataType.BINARY, DataType.MULTILABEL) and not top_k:
        preds = (preds >= threshold).int()
        num_classes = num_classes if not multiclass else 2
    if case == DataType.MULTILABEL and top_k:
        preds = select_topk(preds, top_k)
    if case in (DataType.MULTICLASS, DataType.MULTIDIM_MULTICLASS) or multiclass:
        if preds.is_floating_point():
            num_classes = preds.shape[1]
            preds = select_topk(preds, top_k or 1)
        else:
            num_classes = num_classes or int(max(preds.max().item(), target.max().item()) + 1)
            preds = to_onehot(preds, max(2, num_classes))
        target = to_onehot(target, max(2, num_classes))
        if multiclass is False:
            preds, target = preds[:, 1, ...], target[:, 1, ...]
    if not _empty(preds, target):
        if (case in (DataType.MULTICLASS, DataType.MULTIDIM_MULTICLASS) and multiclass is not False) or multiclass:
            target = target.reshape(target.shape[0], target.shape[1], -1)
            preds = preds.reshape(preds.shape[0], preds.shape[1], -1)
        else:
            target = target.reshape(target.shape[0], -1)
            preds = preds.reshape(preds.shape[0], -1)
    if preds.ndim > 2:
        preds, target = preds.squeeze(-1), target.squeeze(-1)
    return preds.int(), target.int(), case


def _del_column(data: Tensor, idx: int) -> Tensor:
    return torch.cat([data[:, :idx], data[:, (idx + 1):]], 1)


def _drop_negative_ignored_indices(preds: Tensor, target: Tensor, ignore_index: int, mode: DataType):
    if mode == DataType.MULTIDIM_MULTICLASS and preds.dtype == torch.float:
        c = preds.shape[1]
        preds = preds.transpose(1, preds.ndim - 1).reshape(-1, c)
        target = target.reshape(-1)
    if mode in (DataType.MULTICLASS, DataType.MULTIDIM_MULTICLASS):
        keep = target != ignore_index
        preds, target = preds[keep], target[keep]
    return preds, target


def _stat_scores(preds: Tensor, target: Tensor, reduce: Optional[str] = "micro"):
    if reduce == "micro":
        dim: Union[int, List[int]] = [0, 1] if preds.ndim == 2 else [1, 2]
    elif reduce == "macro":
        dim = 0 if preds.ndim == 2 else 2
    else:
        dim = 1
    correct = target == preds
    pos, neg = preds == 1, preds == 0
    tp = (correct & pos).sum(dim=dim)
    fp = (~correct & pos).sum(dim=dim)
    tn = (correct & neg).sum(dim=dim)
    fn = (~correct & neg).sum(dim=dim)
    return tp.long(), fp.long(), tn.long(), fn.long()


def _stat_scores_update(
    preds: Tensor,
    target: Tensor,
    reduce: Optional[str] = "micro",
    mdmc_reduce: Optional[str] = None,
    num_classes: Optional[int] = None,
    top_k: Optional[int] = 1,
    threshold: float = 0.5,
    multiclass: Optional[bool] = None,
    ignore_index: Optional[int] = None,
    mode: Optional[DataType] = None,
):
    dropped = False
    if ignore_index is not None and ignore_index < 0 and mode is not None:
        preds, target = _drop_negative_ignored_indices(preds, target, ignore_index, mode)
        dropped = True
    preds, target, _ = _input_format_classification(
        preds, target, threshold=threshold, num_classes=num_classes, multiclass=multiclass, top_k=top_k,
        ignore_index=ignore_index,
    )
    if ignore_index is not None and ignore_index >= preds.shape[1]:
        raise ValueError(f"The `ignore_index` {ignore_index} is not valid for inputs with {preds.shape[1]} classes")
    if ignore_index is not None and preds.shape[1] == 1:
        raise ValueError("You can not use `ignore_index` with binary data.")
    if preds.ndim == 3:
        if not mdmc_reduce:
            raise ValueError(
                "When your inputs are multi-dimensional multi-class, you have to set the `mdmc_reduce` parameter"
            )
        if mdmc_reduce == "global":
            preds = preds.transpose(1, 2).reshape(-1, preds.shape[1])
            target = target.transpose(1, 2).reshape(-1, target.shape[1])
    if ignore_index is not None and reduce != "macro" and not dropped:
        preds, target = _del_column(preds, ignore_index), _del_column(target, ignore_index)
    tp, fp, tn, fn = _stat_scores(preds, target, reduce=reduce)
    if ignore_index is not None and reduce == "macro" and not dropped:
        for t in (tp, fp, tn, fn):
            t[..., ignore_index] = -1
    return tp, fp, tn, fn


def _reduce_stat_scores(
    numerator: Tensor,
    denominator: Tensor,
    weights: Optional[Tensor],
    average: Optional[str],
    mdmc_average: Optional[str],
    zero_division: int = 0,
) -> Tensor:
    numerator, denominator = numerator.float(), denominator.float()
    zero_div = denominator == 0
    ignore = denominator < 0
    weights = torch.ones_like(denominator) if weights is None else weights.float()
    numerator = torch.where(zero_div, torch.full_like(numerator, float(zero_division)), numerator)
    denominator = torch.where(zero_div | ignore, torch.ones_like(denominator), denominator)
    weights = torch.where(ignore, torch.zeros_like(weights), weights)
    if average not in (AverageMethod.MICRO, AverageMethod.NONE, None):
        weights = weights / weights.sum(dim=-1, keepdim=True)
    scores = weights * (numerator / denominator)
    scores = torch.where(torch.isnan(scores), torch.full_like(scores, float(zero_division)), scores)
    if mdmc_average == MDMCAverageMethod.SAMPLEWISE:
        scores = scores.mean(dim=0)
        ignore = ignore.sum(dim=0).bool()
    if average in (AverageMethod.NONE, None):
        return torch.where(ignore, torch.full_like(scores, float("nan")), scores)
    return scores.sum()
