"""Stat-scores module metrics (parity: reference ``S/classification/stat_scores.py:43-560``).

All classification metrics derived from tp/fp/tn/fn (Accuracy, Precision, Recall, F-beta, Specificity, Hamming,
...) inherit from these classes.  ``update`` runs one fused HIP kernel that accumulates straight into the
``tp/fp/tn/fn`` state tensors in place (global mode) -- no temporaries, no host sync, HIP-graph capturable.
"""
from typing import Any, Callable, List, Optional, Sequence, Tuple, Type, Union

import torch
from torch import Tensor

from torchmetrics_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_amd.functional.classification.stat_scores import (
    _binary_like_stats,
    _binary_stat_scores_arg_validation,
    _binary_stat_scores_compute,
    _binary_stat_scores_tensor_validation,
    _multiclass_stat_scores_arg_validation,
    _multiclass_stat_scores_compute,
    _multiclass_stat_scores_tensor_validation,
    _multiclass_stats,
    _multilabel_stat_scores_arg_validation,
    _multilabel_stat_scores_compute,
    _multilabel_stat_scores_tensor_validation,
    _StatWorkspace,
)
from torchmetrics_amd import ops
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import dim_zero_cat
from torchmetrics_amd.utilities.enums import ClassificationTask
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class _AbstractStatScores(Metric):
    tp: Union[List[Tensor], Tensor]
    fp: Union[List[Tensor], Tensor]
    tn: Union[List[Tensor], Tensor]
    fn: Union[List[Tensor], Tensor]

    # the score of the class's compute() (`_stat_reduce(kind, ...)`); set by the score classes (Accuracy, Precision,
    # ...) -- those get the native forward (csrc/bindings/fastcall.cpp NativeForward, classification/forward.hip)
    _stat_kind: Optional[str] = None

    def _create_state(self, size: int, multidim_average: str = "global") -> None:
        samplewise = multidim_average == "samplewise"
        for name in ("tp", "fp", "tn", "fn"):
            self.add_state(
                name,
                [] if samplewise else torch.zeros(size, dtype=torch.long),
                dist_reduce_fx="cat" if samplewise else "sum",
            )
        self._ws = _StatWorkspace()
        self._install_native_update()
        self._install_native_forward()

    def _native_family(self) -> Optional[type]:
        cls = type(self)
        family = next((c for c in (MulticlassStatScores, MultilabelStatScores, BinaryStatScores) if isinstance(self, c)),
                      None)
        if family is None or cls.update is not family.update or getattr(self, "multidim_average", None) != "global":
            return None
        return family

    def _install_native_update(self) -> None:
        """ROCm: ``update`` = the update kernel + the fold into the states, driven from C++ (csrc/bindings/
        fastcall.cpp ``stats_updater``); inputs off its fast path (CPU, top_k > 1, other shapes / dtypes) run the
        Python ``update``."""
        family = self._native_family()
        if family is None:
            return
        kind = {MulticlassStatScores: ops.FWD_MULTICLASS, MultilabelStatScores: ops.FWD_MULTILABEL,
                BinaryStatScores: ops.FWD_BINARY}[family]
        fast = ops.native_updater("stats", self.__dict__, self.__dict__["update"], kind)
        if fast is not None:
            self.__dict__["update"] = fast

    def _install_native_forward(self) -> None:
        """ROCm: ``forward`` = the update kernel + one fused fold-and-score launch, driven from C++ (the batch value is
        ``compute()``'s own score body on the batch counts).  Only for the classes whose ``compute`` is the plain
        fused score and whose ``update`` / ``forward`` / ``reset`` are the family's own; per-call preconditions
        (global average, top_k = 1, plain input shapes, no dist_sync_on_step, states nobody else holds) are checked
        natively, anything else runs ``Metric.forward``."""
        cls = type(self)
        owner = next((c for c in cls.__mro__ if "_stat_kind" in c.__dict__), None)
        if owner is None or owner.__dict__["_stat_kind"] is None or getattr(self, "multidim_average", None) != "global":
            return
        family = next((c for c in (MulticlassStatScores, MultilabelStatScores, BinaryStatScores) if isinstance(self, c)),
                      None)
        if (family is None or cls.compute is not owner.compute or cls.update is not family.update
                or cls.forward is not Metric.forward or cls.reset is not Metric.reset):
            return
        kind = {MulticlassStatScores: ops.FWD_MULTICLASS, MultilabelStatScores: ops.FWD_MULTILABEL,
                BinaryStatScores: ops.FWD_BINARY}[family]
        fast = ops.native_forward(kind, self.__dict__, Metric.forward.__get__(self, cls), owner.__dict__["_stat_kind"])
        if fast is not None:
            self.__dict__["forward"] = fast

    def _update_state(self, tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor) -> None:
        if self.multidim_average == "samplewise":
            self.tp.append(tp)
            self.fp.append(fp)
            self.tn.append(tn)
            self.fn.append(fn)
        else:
            self.tp += tp
            self.fp += fp
            self.tn += tn
            self.fn += fn

    def _final_state(self) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
        return dim_zero_cat(self.tp), dim_zero_cat(self.fp), dim_zero_cat(self.tn), dim_zero_cat(self.fn)

    # -- fused-path helpers ------------------------------------------------------------------------------------
    def _states_inplace(self, device: torch.device) -> Optional[Tuple[Tensor, Tensor, Tensor, Tensor]]:
        """The global-mode state tensors if they can be accumulated in place by the kernel."""
        if self.multidim_average == "samplewise":
            return None
        st = (self.tp, self.fp, self.tn, self.fn)
        if all(isinstance(s, Tensor) and s.device == device and s.dtype == torch.long and s.is_contiguous() for s in st):
            return st  # type: ignore[return-value]
        return None

    def _flag_for(self, x: Tensor) -> Optional[Tensor]:
        return self._device_error_buffer(x.device) if self.validate_args else None

    def _post_update_check(self, x: Tensor) -> None:
        # CPU inputs: raise immediately (as the reference); GPU: deferred to compute()
        if self.validate_args and not x.is_cuda:
            self._raise_device_errors()

    def _apply(self, fn: Callable, exclude_state: Sequence[str] = "") -> Any:
        this = super()._apply(fn, exclude_state)
        if hasattr(this, "_ws"):
            this._ws = _StatWorkspace()
        return this


class BinaryStatScores(_AbstractStatScores):
    """tp, fp, tn, fn and support for binary tasks."""

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = None
    full_state_update: bool = False

    def __init__(
        self,
        threshold: float = 0.5,
        multidim_average: str = "global",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super(_AbstractStatScores, self).__init__(**kwargs)
        if validate_args:
            _binary_stat_scores_arg_validation(threshold, multidim_average, ignore_index)
        self.threshold = threshold
        self.multidim_average = multidim_average
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_state(size=1, multidim_average=multidim_average)

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _binary_stat_scores_tensor_validation(preds, target, self.multidim_average, self.ignore_index)
        out = self._states_inplace(preds.device)
        res = _binary_like_stats(
            preds, target, 1, self.threshold, self.multidim_average, self.ignore_index, self._flag_for(preds),
            out=out, workspace=self._ws,
        )
        if out is None:
            if self.multidim_average == "samplewise":
                self._update_state(*res)
            else:
                self._update_state(*(r.view(1) for r in res))
        self._post_update_check(preds)

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _binary_stat_scores_compute(tp, fp, tn, fn, self.multidim_average)


class MulticlassStatScores(_AbstractStatScores):
    """tp, fp, tn, fn and support per class for multiclass tasks."""

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = None
    full_state_update: bool = False

    def __init__(
        self,
        num_classes: int,
        top_k: int = 1,
        average: Optional[str] = "macro",
        multidim_average: str = "global",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super(_AbstractStatScores, self).__init__(**kwargs)
        if validate_args:
            _multiclass_stat_scores_arg_validation(num_classes, top_k, average, multidim_average, ignore_index)
        self.num_classes = num_classes
        self.top_k = top_k
        self.average = average
        self.multidim_average = multidim_average
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._micro = average == "micro" and top_k == 1
        self._create_state(size=1 if self._micro else num_classes, multidim_average=multidim_average)

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _multiclass_stat_scores_tensor_validation(
                preds, target, self.num_classes, self.multidim_average, self.ignore_index
            )
        out = self._states_inplace(preds.device)
        res = _multiclass_stats(
            preds, target, self.num_classes, self.top_k, self._micro, self.multidim_average, self.ignore_index,
            self._flag_for(preds), out=out, workspace=self._ws,
        )
        if out is None:
            self._update_state(*res)
        self._post_update_check(preds)

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _multiclass_stat_scores_compute(tp, fp, tn, fn, self.average, self.multidim_average)


class MultilabelStatScores(_AbstractStatScores):
    """tp, fp, tn, fn and support per label for multilabel tasks."""

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = None
    full_state_update: bool = False

    def __init__(
        self,
        num_labels: int,
        threshold: float = 0.5,
        average: Optional[str] = "macro",
        multidim_average: str = "global",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super(_AbstractStatScores, self).__init__(**kwargs)
        if validate_args:
            _multilabel_stat_scores_arg_validation(num_labels, threshold, average, multidim_average, ignore_index)
        self.num_labels = num_labels
        self.threshold = threshold
        self.average = average
        self.multidim_average = multidim_average
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_state(size=num_labels, multidim_average=multidim_average)

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _multilabel_stat_scores_tensor_validation(
                preds, target, self.num_labels, self.multidim_average, self.ignore_index
            )
        out = self._states_inplace(preds.device)
        res = _binary_like_stats(
            preds, target, self.num_labels, self.threshold, self.multidim_average, self.ignore_index,
            self._flag_for(preds), out=out, workspace=self._ws,
        )
        if out is None:
            if self.multidim_average == "samplewise":
                res = tuple(r.view(-1, self.num_labels) for r in res)
            self._update_state(*res)
        self._post_update_check(preds)

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _multilabel_stat_scores_compute(tp, fp, tn, fn, self.average, self.multidim_average)


class StatScores(_ClassificationTaskWrapper):
    """Task wrapper: ``StatScores(task=...)`` returns the Binary/Multiclass/Multilabel variant."""

    def __new__(  # type: ignore[misc]
        cls: Type["StatScores"],
        task: str,
        threshold: float = 0.5,
        num_classes: Optional[int] = None,
        num_labels: Optional[int] = None,
        average: Optional[str] = "micro",
        multidim_average: str = "global",
        top_k: Optional[int] = 1,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> Metric:
        task = ClassificationTask.from_str(task)
        assert multidim_average is not None  # noqa: S101
        kwargs.update({"multidim_average": multidim_average, "ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTask.BINARY:
            return BinaryStatScores(threshold, **kwargs)
        if task == ClassificationTask.MULTICLASS:
            if not isinstance(num_classes, int):
                raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
            if not isinstance(top_k, int):
                raise ValueError(f"`top_k` is expected to be `int` but `{type(top_k)} was passed.`")
            return MulticlassStatScores(num_classes, top_k, average, **kwargs)
        if task == ClassificationTask.MULTILABEL:
            if not isinstance(num_labels, int):
                raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
            return MultilabelStatScores(num_labels, threshold, average, **kwargs)
        raise ValueError(f"Task {task} not supported!")
