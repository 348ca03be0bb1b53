"""Confusion-matrix module metrics and the metrics derived from them (Cohen's kappa, Jaccard, MCC).

Parity: reference ``S/classification/confusion_matrix.py:51-560``, ``cohen_kappa.py``, ``jaccard.py``,
``matthews_corrcoef.py``.  The ``confmat`` state is accumulated *in place* by the HIP kernel on every update, so
``MulticlassConfusionMatrix(1000)`` costs one pass over the ``[N, 1000]`` logits plus N 64-bit atomics per update,
and distributed sync is a single 8 MB RCCL ``all_reduce`` (the reference all_gathers W x 8 MB).
"""
from typing import Any, List, Optional, Type

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_amd.functional.classification.cohen_kappa import (
    _binary_cohen_kappa_arg_validation,
    _cohen_kappa_reduce,
    _multiclass_cohen_kappa_arg_validation,
)
from torchmetrics_amd.functional.classification.confusion_matrix import (
    _binary_confmat_accumulate,
    _binary_confusion_matrix_arg_validation,
    _binary_confusion_matrix_tensor_validation,
    _confusion_matrix_reduce,
    _multiclass_confmat_accumulate,
    _multiclass_confusion_matrix_arg_validation,
    _multiclass_confusion_matrix_tensor_validation,
    _multilabel_confmat_accumulate,
    _multilabel_confusion_matrix_arg_validation,
    _multilabel_confusion_matrix_tensor_validation,
)
from torchmetrics_amd.functional.classification.jaccard import _check_avg, _jaccard_index_reduce
from torchmetrics_amd.functional.classification.matthews_corrcoef import _matthews_corrcoef_reduce
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.enums import ClassificationTask, ClassificationTaskNoMultilabel
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE, plot_confusion_matrix


class _ConfmatBase(Metric):
    confmat: Tensor
    is_differentiable = False
    higher_is_better: Optional[bool] = None
    full_state_update: bool = False

    def _confmat_target(self, device: torch.device) -> Optional[Tensor]:
        cm = self.confmat
        if isinstance(cm, Tensor) and cm.device == device and cm.dtype == torch.long and cm.is_contiguous():
            return cm
        return None

    def _accumulate(self, fn: Any, preds: Tensor, *args: Any) -> None:
        # device checks by index (Tensor.get_device is ~3x cheaper than building and comparing torch.device objects)
        dev = preds.get_device()
        flag = None
        if self.validate_args:
            flag = self._device_errors
            if flag is None or flag.get_device() != dev:
                flag = self._device_error_buffer(preds.device)
        cm = self.confmat
        if isinstance(cm, Tensor) and cm.get_device() == dev and cm.dtype is torch.long and cm.is_contiguous():
            target_cm = cm
        else:
            target_cm = self._confmat_target(preds.device)
        if target_cm is None:
            tmp = torch.zeros_like(self.confmat, dtype=torch.long, device=preds.device)
            fn(preds, *args[:1], tmp, *args[1:], flag)
            self.confmat = self.confmat + tmp.to(self.confmat.device)
        else:
            fn(preds, *args[:1], target_cm, *args[1:], flag)
        if self.validate_args and not preds.is_cuda:
            self._raise_device_errors()

    def _bin_ws(self, n: int, device: torch.device) -> tuple:
        ws = getattr(self, "_cm_ws", None)
        if ws is None or ws[0].numel() != n or ws[0].device != device:
            ws = (torch.zeros(n, dtype=torch.int64, device=device), torch.zeros(1, dtype=torch.int32, device=device))
            self._cm_ws = ws
        return ws

    def plot(
        self,
        val: Optional[Tensor] = None,
        ax: Optional[_AX_TYPE] = None,
        add_text: bool = True,
        labels: Optional[List[str]] = None,
        cmap: Optional[Any] = None,
    ) -> _PLOT_OUT_TYPE:
        val = val if val is not None else self.compute()
        if not isinstance(val, Tensor):
            raise TypeError(f"Expected val to be a single tensor but got {val}")
        return plot_confusion_matrix(val, ax=ax, add_text=add_text, labels=labels, cmap=cmap)


class BinaryConfusionMatrix(_ConfmatBase):
    """``[2, 2]`` confusion matrix for binary tasks."""

    def __init__(
        self,
        threshold: float = 0.5,
        ignore_index: Optional[int] = None,
        normalize: Optional[str] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _binary_confusion_matrix_arg_validation(threshold, ignore_index, normalize)
        self.threshold = threshold
        self.ignore_index = ignore_index
        self.normalize = normalize
        self.validate_args = validate_args
        self.add_state("confmat", torch.zeros(2, 2, dtype=torch.long), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _binary_confusion_matrix_tensor_validation(preds, target, self.ignore_index)
        ws = self._bin_ws(7, preds.device)
        self._accumulate(
            lambda p, t, cm, thr, ii, flag: _binary_confmat_accumulate(p, t, cm, thr, ii, flag, ws),
            preds, target, self.threshold, self.ignore_index,
        )

    def compute(self) -> Tensor:
        return _confusion_matrix_reduce(self.confmat, self.normalize)


class MulticlassConfusionMatrix(_ConfmatBase):
    """``[C, C]`` confusion matrix for multiclass tasks."""

    def __init__(
        self,
        num_classes: int,
        ignore_index: Optional[int] = None,
        normalize: Optional[str] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multiclass_confusion_matrix_arg_validation(num_classes, ignore_index, normalize)
        self.num_classes = num_classes
        self.ignore_index = ignore_index
        self.normalize = normalize
        self.validate_args = validate_args
        self.add_state("confmat", torch.zeros(num_classes, num_classes, dtype=torch.long), dist_reduce_fx="sum")
        self._install_native_update()
        self._install_native_forward()

    def _install_native_forward(self) -> None:
        """ROCm: ``forward`` = zeros(C, C) + the update kernel into it + one add into the global matrix, driven from C++
        (csrc/bindings/fastcall.cpp NativeForward); only for this class's own update / compute / forward / reset."""
        cls = type(self)
        if (cls.update is not MulticlassConfusionMatrix.update or cls.compute is not MulticlassConfusionMatrix.compute
                or cls.forward is not Metric.forward or cls.reset is not Metric.reset):
            return
        fast = ops.native_forward(ops.FWD_CONFMAT, self.__dict__, Metric.forward.__get__(self, cls))
        if fast is not None:
            self.__dict__["forward"] = fast

    def _install_native_update(self) -> None:
        """``update`` becomes ONE native call on ROCm (csrc/bindings/fastcall.cpp ``confmat_updater``): the shape /
        dtype checks, the ``_update_count`` / ``_computed`` bookkeeping and the kernel launch without a Python frame;
        any other input goes through the Python ``update`` below.  A subclass that overrides ``update`` keeps its own
        (the native call would bypass it)."""
        if type(self).update is not MulticlassConfusionMatrix.update:
            return
        fast = ops.native_updater("confmat", self.__dict__, self.__dict__["update"])
        if fast is not None:
            self.__dict__["update"] = fast

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _multiclass_confusion_matrix_tensor_validation(preds, target, self.num_classes, self.ignore_index)
        self._accumulate(_multiclass_confmat_accumulate, preds, target, self.num_classes, self.ignore_index)

    def compute(self) -> Tensor:
        return _confusion_matrix_reduce(self.confmat, self.normalize)


class MultilabelConfusionMatrix(_ConfmatBase):
    """``[L, 2, 2]`` confusion matrices for multilabel tasks."""

    def __init__(
        self,
        num_labels: int,
        threshold: float = 0.5,
        ignore_index: Optional[int] = None,
        normalize: Optional[str] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multilabel_confusion_matrix_arg_validation(num_labels, threshold, ignore_index, normalize)
        self.num_labels = num_labels
        self.threshold = threshold
        self.ignore_index = ignore_index
        self.normalize = normalize
        self.validate_args = validate_args
        self.add_state("confmat", torch.zeros(num_labels, 2, 2, dtype=torch.long), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _multilabel_confusion_matrix_tensor_validation(preds, target, self.num_labels, self.ignore_index)
        ws = self._bin_ws(7 * self.num_labels, preds.device)
        self._accumulate(
            lambda p, t, cm, nl, thr, ii, flag: _multilabel_confmat_accumulate(p, t, cm, nl, thr, ii, flag, ws),
            preds, target, self.num_labels, self.threshold, self.ignore_index,
        )

    def compute(self) -> Tensor:
        return _confusion_matrix_reduce(self.confmat, self.normalize)


class ConfusionMatrix(_ClassificationTaskWrapper):
    def __new__(  # type: ignore[misc]
        cls: Type["ConfusionMatrix"],
        task: str,
        threshold: float = 0.5,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        normalize: Optional[str] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        task = ClassificationTask.from_str(task)
        kwargs.update({"normalize": normalize, "ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTask.BINARY:
            return BinaryConfusionMatrix(threshold, **kwargs)
        if task == ClassificationTask.MULTICLASS:
            if not isinstance(num_classes, int):
                raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
            return MulticlassConfusionMatrix(num_classes, **kwargs)
        if task == ClassificationTask.MULTILABEL:
            if not isinstance(num_labels, int):
                raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
            return MultilabelConfusionMatrix(num_labels, threshold, **kwargs)
        raise ValueError(f"Task {task} not supported!")


# --------------------------------------------------------------------------------------------------- Cohen kappa
class BinaryCohenKappa(BinaryConfusionMatrix):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        threshold: float = 0.5,
        ignore_index: Optional[int] = None,
        weights: Optional[str] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(threshold, ignore_index, normalize=None, validate_args=False, **kwargs)
        if validate_args:
            _binary_cohen_kappa_arg_validation(threshold, ignore_index, weights)
        self.weights = weights
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        return _cohen_kappa_reduce(self.confmat, self.weights)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        return self._plot(val, ax)


class MulticlassCohenKappa(MulticlassConfusionMatrix):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def __init__(
        self,
        num_classes: int,
        ignore_index: Optional[int] = None,
        weights: Optional[str] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(num_classes, ignore_index, normalize=None, validate_args=False, **kwargs)
        if validate_args:
            _multiclass_cohen_kappa_arg_validation(num_classes, ignore_index, weights)
        self.weights = weights
        self.validate_args = validate_args

    def compute(self) -> Tensor:
        return _cohen_kappa_reduce(self.confmat, self.weights)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        return self._plot(val, ax)


class CohenKappa(_ClassificationTaskWrapper):
    def __new__(  # type: ignore[misc]
        cls: Type["CohenKappa"],
        task: str,
        threshold: float = 0.5,
        num_classes: Optional[int] = None,
        weights: Optional[str] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        task = ClassificationTaskNoMultilabel.from_str(task)
        kwargs.update({"weights": weights, "ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTaskNoMultilabel.BINARY:
            return BinaryCohenKappa(threshold, **kwargs)
        if task == ClassificationTaskNoMultilabel.MULTICLASS:
            if not isinstance(num_classes, int):
                raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
            return MulticlassCohenKappa(num_classes, **kwargs)
        raise ValueError(f"Task {task} not supported!")


# ------------------------------------------------------------------------------------------------------- Jaccard
class BinaryJaccardIndex(BinaryConfusionMatrix):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, threshold: float = 0.5, ignore_index: Optional[int] = None, validate_args: bool = True,
                 **kwargs: Any) -> None:
        super().__init__(threshold=threshold, ignore_index=ignore_index, normalize=None, validate_args=validate_args,
                         **kwargs)

    def compute(self) -> Tensor:
        return _jaccard_index_reduce(self.confmat, average="binary")

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        return self._plot(val, ax)


class MulticlassJaccardIndex(MulticlassConfusionMatrix):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def __init__(self, num_classes: int, average: Optional[str] = "macro", ignore_index: Optional[int] = None,
                 validate_args: bool = True, **kwargs: Any) -> None:
        super().__init__(num_classes=num_classes, ignore_index=ignore_index, normalize=None,
                         validate_args=False, **kwargs)
        if validate_args:
            _multiclass_confusion_matrix_arg_validation(num_classes, ignore_index)
            _check_avg(average)
        self.validate_args = validate_args
        self.average = average

    def compute(self) -> Tensor:
        return _jaccard_index_reduce(self.confmat, average=self.average, ignore_index=self.ignore_index)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        return self._plot(val, ax)


class MultilabelJaccardIndex(MultilabelConfusionMatrix):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Label"

    def __init__(self, num_labels: int, threshold: float = 0.5, average: Optional[str] = "macro",
                 ignore_index: Optional[int] = None, validate_args: bool = True, **kwargs: Any) -> None:
        super().__init__(num_labels=num_labels, threshold=threshold, ignore_index=ignore_index, normalize=None,
                         validate_args=False, **kwargs)
        if validate_args:
            _multilabel_confusion_matrix_arg_validation(num_labels, threshold, ignore_index)
            _check_avg(average)
        self.validate_args = validate_args
        self.average = average

    def compute(self) -> Tensor:
        return _jaccard_index_reduce(self.confmat, average=self.average, ignore_index=self.ignore_index)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        return self._plot(val, ax)


class JaccardIndex(_ClassificationTaskWrapper):
    def __new__(  # type: ignore[misc]
        cls: Type["JaccardIndex"],
        task: str,
        threshold: float = 0.5,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        average: Optional[str] = "macro",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        task = ClassificationTask.from_str(task)
        kwargs.update({"ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTask.BINARY:
            return BinaryJaccardIndex(threshold, **kwargs)
        if task == ClassificationTask.MULTICLASS:
            if not isinstance(num_classes, int):
                raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
            return MulticlassJaccardIndex(num_classes, average, **kwargs)
        if task == ClassificationTask.MULTILABEL:
            if not isinstance(num_labels, int):
                raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
            return MultilabelJaccardIndex(num_labels, threshold, average, **kwargs)
        raise ValueError(f"Task {task} not supported!")


# ----------------------------------------------------------------------------------------------------------- MCC
class BinaryMatthewsCorrCoef(BinaryConfusionMatrix):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: Optional[float] = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, threshold: float = 0.5, ignore_index: Optional[int] = None, validate_args: bool = True,
                 **kwargs: Any) -> None:
        super().__init__(threshold, ignore_index, normalize=None, validate_args=validate_args, **kwargs)

    def compute(self) -> Tensor:
        return _matthews_corrcoef_reduce(self.confmat)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        return self._plot(val, ax)


class MulticlassMatthewsCorrCoef(MulticlassConfusionMatrix):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: Optional[float] = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def __init__(self, num_classes: int, ignore_index: Optional[int] = None, validate_args: bool = True,
                 **kwargs: Any) -> None:
        super().__init__(num_classes, ignore_index, normalize=None, validate_args=validate_args, **kwargs)

    def compute(self) -> Tensor:
        return _matthews_corrcoef_reduce(self.confmat)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        return self._plot(val, ax)


class MultilabelMatthewsCorrCoef(MultilabelConfusionMatrix):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: Optional[float] = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Label"

    def __init__(self, num_labels: int, threshold: float = 0.5, ignore_index: Optional[int] = None,
                 validate_args: bool = True, **kwargs: Any) -> None:
        super().__init__(num_labels, threshold, ignore_index, normalize=None, validate_args=validate_args, **kwargs)

    def compute(self) -> Tensor:
        return _matthews_corrcoef_reduce(self.confmat)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:  # type: ignore[override]
        return self._plot(val, ax)


class MatthewsCorrCoef(_ClassificationTaskWrapper):
    def __new__(  # type: ignore[misc]
        cls: Type["MatthewsCorrCoef"],
        task: str,
        threshold: float = 0.5,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        task = ClassificationTask.from_str(task)
        kwargs.update({"ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTask.BINARY:
            return BinaryMatthewsCorrCoef(threshold, **kwargs)
        if task == ClassificationTask.MULTICLASS:
            if not isinstance(num_classes, int):
                raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
            return MulticlassMatthewsCorrCoef(num_classes, **kwargs)
        if task == ClassificationTask.MULTILABEL:
            if not isinstance(num_labels, int):
                raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
            return MultilabelMatthewsCorrCoef(num_labels, threshold, **kwargs)
        raise ValueError(f"Task {task} not supported!")
