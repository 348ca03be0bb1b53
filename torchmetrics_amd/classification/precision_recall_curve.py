"""Curve-family module metrics: PR curve, ROC, AUROC, average precision (+ the shared binned-state base).

Parity: reference ``S/classification/precision_recall_curve.py:55-700``, ``roc.py``, ``auroc.py``,
``average_precision.py``.  With ``thresholds`` set, ``update`` runs the HIP multi-threshold histogram kernel that
accumulates straight into the ``confmat`` state (``[T, 2, 2]`` / ``[T, C, 2, 2]``) with no host sync; with
``thresholds=None`` the (device-side formatted) scores are kept in ``cat`` list states.

Deliberate difference: ``MulticlassPrecisionRecallCurve(average="micro", thresholds=...)`` keeps a ``[T, 2, 2]``
state (the reference declares ``[T, C, 2, 2]`` and broadcasts a ``[T, 2, 2]`` update into it).
"""
from typing import Any, Callable, List, Optional, Sequence, Tuple, Type, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_amd.functional.classification.auroc import (
    _binary_auroc_arg_validation,
    _binary_auroc_compute,
    _multiclass_auroc_arg_validation,
    _multiclass_auroc_compute,
    _multilabel_auroc_arg_validation,
    _multilabel_auroc_compute,
    _reduce_auroc,
)
from torchmetrics_amd.functional.classification.average_precision import (
    _binary_average_precision_compute,
    _multiclass_average_precision_arg_validation,
    _multiclass_average_precision_compute,
    _multilabel_average_precision_arg_validation,
    _multilabel_average_precision_compute,
)
from torchmetrics_amd.functional.classification.precision_recall_curve import (
    Thresholds,
    _adjust_threshold_arg,
    _binary_precision_recall_curve_arg_validation,
    _binary_precision_recall_curve_compute,
    _binary_precision_recall_curve_format,
    _binary_precision_recall_curve_tensor_validation,
    _binned_update,
    _CurveWorkspace,
    _multiclass_precision_recall_curve_arg_validation,
    _multiclass_precision_recall_curve_compute,
    _multiclass_precision_recall_curve_format,
    _multiclass_precision_recall_curve_tensor_validation,
    _multilabel_precision_recall_curve_arg_validation,
    _multilabel_precision_recall_curve_compute,
    _multilabel_precision_recall_curve_format,
    _multilabel_precision_recall_curve_tensor_validation,
)
from torchmetrics_amd.functional.classification.roc import (
    _binary_roc_compute,
    _multiclass_roc_compute,
    _multilabel_roc_compute,
)
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.compute import _auc_compute_without_check
from torchmetrics_amd.utilities.data import dim_zero_cat
from torchmetrics_amd.utilities.enums import ClassificationTask
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE, plot_curve


class _CurveBase(Metric):
    """Shared state handling: ``confmat`` (binned, summed) or ``preds``/``target`` lists (unbinned, cat)."""

    _fold_cat_lists = True  # unbinned compute() only concatenates the preds / target lists

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = None
    full_state_update: bool = False
    preds: List[Tensor]
    target: List[Tensor]
    confmat: Tensor

    def _init_curve_state(self, thresholds: Thresholds, state_shape: Tuple[int, ...]) -> None:
        thresholds = _adjust_threshold_arg(thresholds)
        if thresholds is None:
            self.thresholds = None
            self.add_state("preds", default=[], dist_reduce_fx="cat")
            self.add_state("target", default=[], dist_reduce_fx="cat")
        else:
            self.register_buffer("thresholds", thresholds, persistent=False)
            self.add_state(
                "confmat", default=torch.zeros(len(thresholds), *state_shape, dtype=torch.long), dist_reduce_fx="sum"
            )
        self._cws = _CurveWorkspace()

    def _binned_gpu(self, preds: Tensor) -> bool:
        return self.thresholds is not None and preds.is_cuda

    def _accumulate(self, preds: Tensor, target: Tensor, mode: int, micro: bool = False) -> None:
        st = self.confmat
        inplace = isinstance(st, Tensor) and st.device == preds.device and st.is_contiguous()
        flag = self._device_error_buffer(preds.device) if self.validate_args else None
        res = _binned_update(
            preds, target, self.thresholds, mode, self.ignore_index, micro,
            state=st if inplace else None, err=flag, workspace=self._cws,
        )
        if not inplace:
            self.confmat += res.to(st.device)
        if self.validate_args and not preds.is_cuda:
            self._raise_device_errors()

    def _append(self, preds: Tensor, target: Tensor) -> None:
        self.preds.append(preds)
        self.target.append(target)

    def _state(self) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        return (dim_zero_cat(self.preds), dim_zero_cat(self.target)) if self.thresholds is None else self.confmat

    def _apply(self, fn: Callable, exclude_state: Sequence[str] = "") -> Any:
        this = super()._apply(fn, exclude_state)
        this._cws = _CurveWorkspace()
        return this

    def _plot_curve(self, curve: Any, score: Any, ax: Optional[_AX_TYPE], labels: Tuple[str, str], swap: bool,
                    score_fn: Callable) -> _PLOT_OUT_TYPE:
        curve_computed = curve or self.compute()
        if swap:
            curve_computed = (curve_computed[1], curve_computed[0], curve_computed[2])
        score = score_fn(curve_computed) if not curve and score is True else None
        return plot_curve(curve_computed, score=score, ax=ax, label_names=labels, name=self.__class__.__name__)


# -------------------------------------------------------------------------------------------------- PR curves
class BinaryPrecisionRecallCurve(_CurveBase):
    """Precision-recall pairs at every threshold for binary tasks."""

    def __init__(
        self,
        thresholds: Thresholds = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._init_curve_state(thresholds, (2, 2))

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _binary_precision_recall_curve_tensor_validation(
                preds, target, self.ignore_index, check_values=not self._binned_gpu(preds)
            )
        if self.thresholds is None:
            p, t, _ = _binary_precision_recall_curve_format(preds, target, None, self.ignore_index)
            self._append(p, t)
        else:
            self._accumulate(preds, target, ops.CURVE_BINARY)

    def compute(self) -> Tuple[Tensor, Tensor, Tensor]:
        return _binary_precision_recall_curve_compute(self._state(), self.thresholds)

    def plot(self, curve: Optional[Tuple[Tensor, Tensor, Tensor]] = None, score: Optional[Union[Tensor, bool]] = None,
             ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot_curve(curve, score, ax, ("Recall", "Precision"), True,
                                lambda c: _auc_compute_without_check(c[0], c[1], 1.0))


class MulticlassPrecisionRecallCurve(_CurveBase):
    """One-vs-rest precision-recall curves for multiclass tasks."""

    def __init__(
        self,
        num_classes: int,
        thresholds: Thresholds = None,
        average: Optional[Literal["micro", "macro"]] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index, average)
        self.num_classes = num_classes
        self.average = average
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._init_curve_state(thresholds, (2, 2) if average == "micro" else (num_classes, 2, 2))

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _multiclass_precision_recall_curve_tensor_validation(
                preds, target, self.num_classes, self.ignore_index, check_values=not self._binned_gpu(preds)
            )
        if self.thresholds is None:
            p, t, _ = _multiclass_precision_recall_curve_format(
                preds, target, self.num_classes, None, self.ignore_index, self.average
            )
            self._append(p, t)
        else:
            self._accumulate(preds, target, ops.CURVE_MULTICLASS, micro=self.average == "micro")

    def compute(self) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
        return _multiclass_precision_recall_curve_compute(self._state(), self.num_classes, self.thresholds,
                                                          self.average)

    def plot(self, curve: Any = None, score: Optional[Union[Tensor, bool]] = None,
             ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot_curve(curve, score, ax, ("Recall", "Precision"), True,
                                lambda c: _reduce_auroc(c[0], c[1], average=None))


class MultilabelPrecisionRecallCurve(_CurveBase):
    """Per-label precision-recall curves for multilabel tasks."""

    def __init__(
        self,
        num_labels: int,
        thresholds: Thresholds = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
        self.num_labels = num_labels
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._init_curve_state(thresholds, (num_labels, 2, 2))

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _multilabel_precision_recall_curve_tensor_validation(
                preds, target, self.num_labels, self.ignore_index, check_values=not self._binned_gpu(preds)
            )
        if self.thresholds is None:
            p, t, _ = _multilabel_precision_recall_curve_format(preds, target, self.num_labels, None,
                                                                self.ignore_index)
            self._append(p, t)
        else:
            self._accumulate(preds, target, ops.CURVE_MULTILABEL)

    def compute(self) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
        return _multilabel_precision_recall_curve_compute(self._state(), self.num_labels, self.thresholds,
                                                          self.ignore_index)

    def plot(self, curve: Any = None, score: Optional[Union[Tensor, bool]] = None,
             ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot_curve(curve, score, ax, ("Recall", "Precision"), True,
                                lambda c: _reduce_auroc(c[0], c[1], average=None))


# ------------------------------------------------------------------------------------------------------- ROC
class BinaryROC(BinaryPrecisionRecallCurve):
    """Receiver operating characteristic for binary tasks: ``(fpr, tpr, thresholds)``."""

    plot_upper_bound: Optional[float] = 1.0
    plot_lower_bound: Optional[float] = 0.0
    def compute(self) -> Tuple[Tensor, Tensor, Tensor]:
        return _binary_roc_compute(self._state(), self.thresholds)

    def plot(self, curve: Optional[Tuple[Tensor, Tensor, Tensor]] = None, score: Optional[Union[Tensor, bool]] = None,
             ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot_curve(curve, score, ax, ("False positive rate", "True positive rate"), False,
                                lambda c: _auc_compute_without_check(c[0], c[1], 1.0))


class MulticlassROC(MulticlassPrecisionRecallCurve):
    """One-vs-rest ROC curves for multiclass tasks."""

    plot_legend_name: Optional[str] = 'Class'
    plot_upper_bound: Optional[float] = 1.0
    plot_lower_bound: Optional[float] = 0.0
    def compute(self) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
        return _multiclass_roc_compute(self._state(), self.num_classes, self.thresholds, self.average)

    def plot(self, curve: Any = None, score: Optional[Union[Tensor, bool]] = None,
             ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot_curve(curve, score, ax, ("False positive rate", "True positive rate"), False,
                                lambda c: _reduce_auroc(c[0], c[1], average=None))


class MultilabelROC(MultilabelPrecisionRecallCurve):
    """Per-label ROC curves for multilabel tasks."""

    plot_legend_name: Optional[str] = 'Label'
    plot_upper_bound: Optional[float] = 1.0
    plot_lower_bound: Optional[float] = 0.0
    def compute(self) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
        return _multilabel_roc_compute(self._state(), self.num_labels, self.thresholds, self.ignore_index)

    def plot(self, curve: Any = None, score: Optional[Union[Tensor, bool]] = None,
             ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot_curve(curve, score, ax, ("False positive rate", "True positive rate"), False,
                                lambda c: _reduce_auroc(c[0], c[1], average=None))


# ----------------------------------------------------------------------------------------------------- AUROC
class BinaryAUROC(BinaryPrecisionRecallCurve):
    """Area under the ROC curve for binary tasks (optionally McClish-standardised partial AUC)."""

    higher_is_better: Optional[bool] = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        max_fpr: Optional[float] = None,
        thresholds: Thresholds = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(thresholds=thresholds, ignore_index=ignore_index, validate_args=False, **kwargs)
        if validate_args:
            _binary_auroc_arg_validation(max_fpr, thresholds, ignore_index)
        self.max_fpr = max_fpr
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        return _binary_auroc_compute(self._state(), self.thresholds, self.max_fpr)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MulticlassAUROC(MulticlassPrecisionRecallCurve):
    """One-vs-rest AUROC for multiclass tasks, reduced by ``average``."""

    higher_is_better: Optional[bool] = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def __init__(
        self,
        num_classes: int,
        average: Optional[Literal["macro", "weighted", "none"]] = "macro",
        thresholds: Thresholds = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(
            num_classes=num_classes, thresholds=thresholds, ignore_index=ignore_index, validate_args=False, **kwargs
        )
        if validate_args:
            _multiclass_auroc_arg_validation(num_classes, average, thresholds, ignore_index)
        self.average = average  # type: ignore[assignment]
        self.validate_args = validate_args

    def update(self, preds: Tensor, target: Tensor) -> None:
        # the curve state never uses micro averaging here (a transient toggle through __dict__: no re-versioning)
        d = self.__dict__
        avg, d["average"] = d["average"], None
        try:
            super().update(preds, target)
        finally:
            d["average"] = avg

    def compute(self) -> Tensor:
        return _multiclass_auroc_compute(self._state(), self.num_classes, self.average, self.thresholds)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MultilabelAUROC(MultilabelPrecisionRecallCurve):
    """Per-label AUROC for multilabel tasks, reduced by ``average``."""

    higher_is_better: Optional[bool] = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Label"

    def __init__(
        self,
        num_labels: int,
        average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
        thresholds: Thresholds = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(
            num_labels=num_labels, thresholds=thresholds, ignore_index=ignore_index, validate_args=False, **kwargs
        )
        if validate_args:
            _multilabel_auroc_arg_validation(num_labels, average, thresholds, ignore_index)
        self.average = average
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        return _multilabel_auroc_compute(self._state(), self.num_labels, self.average, self.thresholds,
                                         self.ignore_index)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


# ----------------------------------------------------------------------------------------- average precision
class BinaryAveragePrecision(BinaryPrecisionRecallCurve):
    """Average precision (step-wise area under the PR curve) for binary tasks."""

    higher_is_better: Optional[bool] = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def compute(self) -> Tensor:
        return _binary_average_precision_compute(self._state(), self.thresholds)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MulticlassAveragePrecision(MulticlassPrecisionRecallCurve):
    """One-vs-rest average precision for multiclass tasks."""

    higher_is_better: Optional[bool] = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def __init__(
        self,
        num_classes: int,
        average: Optional[Literal["macro", "weighted", "none"]] = "macro",
        thresholds: Thresholds = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(
            num_classes=num_classes, thresholds=thresholds, ignore_index=ignore_index, validate_args=False, **kwargs
        )
        if validate_args:
            _multiclass_average_precision_arg_validation(num_classes, average, thresholds, ignore_index)
        self.average = average  # type: ignore[assignment]
        self.validate_args = validate_args

    def update(self, preds: Tensor, target: Tensor) -> None:
        # the curve update must not see `average` (micro would flatten the states); a transient toggle through
        # __dict__, so it is no configuration change (Metric.__setattr__ would re-version the metric every update)
        d = self.__dict__
        avg, d["average"] = d["average"], None
        try:
            super().update(preds, target)
        finally:
            d["average"] = avg

    def compute(self) -> Tensor:
        return _multiclass_average_precision_compute(self._state(), self.num_classes, self.average, self.thresholds)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MultilabelAveragePrecision(MultilabelPrecisionRecallCurve):
    """Per-label average precision for multilabel tasks."""

    higher_is_better: Optional[bool] = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Label"

    def __init__(
        self,
        num_labels: int,
        average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
        thresholds: Thresholds = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(
            num_labels=num_labels, thresholds=thresholds, ignore_index=ignore_index, validate_args=False, **kwargs
        )
        if validate_args:
            _multilabel_average_precision_arg_validation(num_labels, average, thresholds, ignore_index)
        self.average = average
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        return _multilabel_average_precision_compute(self._state(), self.num_labels, self.average, self.thresholds,
                                                     self.ignore_index)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


# ----------------------------------------------------------------------------------------------- task wrappers
def _curve_task(binary_cls, multiclass_cls, multilabel_cls, task, num_classes, num_labels, kwargs, mc_extra=None,
                ml_extra=None, bin_extra=None):
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_cls(**(bin_extra or {}), **kwargs)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_cls(num_classes, **(mc_extra or {}), **kwargs)
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_cls(num_labels, **(ml_extra or {}), **kwargs)
    raise ValueError(f"Task {task} not supported!")


class PrecisionRecallCurve(_ClassificationTaskWrapper):
    """Task wrapper: ``PrecisionRecallCurve(task=..., ...)`` returns the task-specific curve metric."""

    def __new__(  # type: ignore[misc]
        cls: Type["PrecisionRecallCurve"],
        task: Literal["binary", "multiclass", "multilabel"],
        thresholds: Thresholds = None,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        kwargs.update({"thresholds": thresholds, "ignore_index": ignore_index, "validate_args": validate_args})
        return _curve_task(BinaryPrecisionRecallCurve, MulticlassPrecisionRecallCurve, MultilabelPrecisionRecallCurve,
                           task, num_classes, num_labels, kwargs)


class ROC(_ClassificationTaskWrapper):
    """Task wrapper: ``ROC(task=..., ...)`` returns the task-specific ROC metric."""

    def __new__(  # type: ignore[misc]
        cls: Type["ROC"],
        task: Literal["binary", "multiclass", "multilabel"],
        thresholds: Thresholds = None,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        kwargs.update({"thresholds": thresholds, "ignore_index": ignore_index, "validate_args": validate_args})
        return _curve_task(BinaryROC, MulticlassROC, MultilabelROC, task, num_classes, num_labels, kwargs)


class AUROC(_ClassificationTaskWrapper):
    """Task wrapper: ``AUROC(task=..., ...)`` returns the task-specific AUROC metric."""

    def __new__(  # type: ignore[misc]
        cls: Type["AUROC"],
        task: Literal["binary", "multiclass", "multilabel"],
        thresholds: Thresholds = None,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        average: Optional[Literal["macro", "weighted", "none"]] = "macro",
        max_fpr: Optional[float] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        kwargs.update({"thresholds": thresholds, "ignore_index": ignore_index, "validate_args": validate_args})
        return _curve_task(BinaryAUROC, MulticlassAUROC, MultilabelAUROC, task, num_classes, num_labels, kwargs,
                           mc_extra={"average": average}, ml_extra={"average": average},
                           bin_extra={"max_fpr": max_fpr})


class AveragePrecision(_ClassificationTaskWrapper):
    """Task wrapper: ``AveragePrecision(task=..., ...)`` returns the task-specific average precision metric."""

    def __new__(  # type: ignore[misc]
        cls: Type["AveragePrecision"],
        task: Literal["binary", "multiclass", "multilabel"],
        thresholds: Thresholds = None,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        average: Optional[Literal["macro", "weighted", "none"]] = "macro",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        kwargs.update({"thresholds": thresholds, "ignore_index": ignore_index, "validate_args": validate_args})
        return _curve_task(BinaryAveragePrecision, MulticlassAveragePrecision, MultilabelAveragePrecision, task,
                           num_classes, num_labels, kwargs, mc_extra={"average": average},
                           ml_extra={"average": average})
