"""F-beta / F1 module metrics. Parity: reference ``S/classification/f_beta.py``.

Thin subclasses of the fused stat-scores metrics: ``update`` is the shared HIP kernel, ``compute`` is the score
algebra of :mod:`torchmetrics_amd.functional.classification._reductions`.
"""
from typing import Any, Optional, Sequence, Type, Union

from torch import Tensor

from torchmetrics_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_amd.classification.stat_scores import BinaryStatScores, MulticlassStatScores, MultilabelStatScores
from torchmetrics_amd.functional.classification._family import _check_beta
from torchmetrics_amd.functional.classification._reductions import _stat_reduce
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.enums import ClassificationTask
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class BinaryFBetaScore(BinaryStatScores):
    """Binary F-beta."""

    is_differentiable = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        beta: float,
        threshold: float = 0.5,
        multidim_average: str = "global",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(threshold=threshold, multidim_average=multidim_average, ignore_index=ignore_index,
                         validate_args=False, **kwargs)
        if validate_args:
            _check_beta(beta)
            from torchmetrics_amd.functional.classification.stat_scores import _binary_stat_scores_arg_validation

            _binary_stat_scores_arg_validation(threshold, multidim_average, ignore_index)
        self.validate_args = validate_args
        self.beta = beta

    _stat_kind = "fbeta"  # compute() is the fused `_stat_reduce` score: native forward applies

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _stat_reduce("fbeta", tp, fp, tn, fn, "binary", self.multidim_average, beta=self.beta)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MulticlassFBetaScore(MulticlassStatScores):
    """Multiclass F-beta."""

    is_differentiable = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def __init__(
        self,
        beta: float,
        num_classes: int,
        top_k: int = 1,
        average: Optional[str] = "macro",
        multidim_average: str = "global",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(num_classes=num_classes, top_k=top_k, average=average, multidim_average=multidim_average,
                         ignore_index=ignore_index, validate_args=validate_args, **kwargs)
        if validate_args:
            _check_beta(beta)
        self.beta = beta

    _stat_kind = "fbeta"  # compute() is the fused `_stat_reduce` score: native forward applies

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _stat_reduce("fbeta", tp, fp, tn, fn, self.average, self.multidim_average, beta=self.beta)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MultilabelFBetaScore(MultilabelStatScores):
    """Multilabel F-beta."""

    is_differentiable = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Label"

    def __init__(
        self,
        beta: float,
        num_labels: int,
        threshold: float = 0.5,
        average: Optional[str] = "macro",
        multidim_average: str = "global",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(num_labels=num_labels, threshold=threshold, average=average,
                         multidim_average=multidim_average, ignore_index=ignore_index, validate_args=validate_args,
                         **kwargs)
        if validate_args:
            _check_beta(beta)
        self.beta = beta

    _stat_kind = "fbeta"  # compute() is the fused `_stat_reduce` score: native forward applies

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _stat_reduce("fbeta", tp, fp, tn, fn, self.average, self.multidim_average, multilabel=True, beta=self.beta)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class BinaryF1Score(BinaryFBetaScore):
    """Binary F1."""

    is_differentiable = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        threshold: float = 0.5,
        multidim_average: str = "global",
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(1.0, threshold, multidim_average, ignore_index, validate_args, **kwargs)

    _stat_kind = "fbeta"  # compute() is the fused `_stat_reduce` score: native forward applies

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _stat_reduce("fbeta", tp, fp, tn, fn, "binary", self.multidim_average, beta=self.beta)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MulticlassF1Score(MulticlassFBetaScore):
    """Multiclass F1."""

    is_differentiable = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

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
        super().__init__(1.0, num_classes, top_k=top_k, average=average, multidim_average=multidim_average,
                         ignore_index=ignore_index, validate_args=validate_args, **kwargs)

    _stat_kind = "fbeta"  # compute() is the fused `_stat_reduce` score: native forward applies

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _stat_reduce("fbeta", tp, fp, tn, fn, self.average, self.multidim_average, beta=self.beta)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MultilabelF1Score(MultilabelFBetaScore):
    """Multilabel F1."""

    is_differentiable = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Label"

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
        super().__init__(1.0, num_labels, threshold, average, multidim_average, ignore_index, validate_args, **kwargs)

    _stat_kind = "fbeta"  # compute() is the fused `_stat_reduce` score: native forward applies

    def compute(self) -> Tensor:
        tp, fp, tn, fn = self._final_state()
        return _stat_reduce("fbeta", tp, fp, tn, fn, self.average, self.multidim_average, multilabel=True, beta=self.beta)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class FBetaScore(_ClassificationTaskWrapper):
    """Task wrapper: returns Binary/Multiclass/MultilabelFBetaScore for ``task``."""

    def __new__(  # type: ignore[misc]
        cls: Type["FBetaScore"],
        task: str,
        beta: float = 1.0,
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
        kwargs.update({"multidim_average": multidim_average, "ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTask.BINARY:
            return BinaryFBetaScore(beta, threshold, **kwargs)
        if task == ClassificationTask.MULTICLASS:
            if not isinstance(num_classes, int):
                raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
            if not isinstance(top_k, int):
                raise ValueError(f"`top_k` is expected to be `int` but `{type(top_k)} was passed.`")
            return MulticlassFBetaScore(beta, num_classes, top_k, average, **kwargs)
        if task == ClassificationTask.MULTILABEL:
            if not isinstance(num_labels, int):
                raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
            return MultilabelFBetaScore(beta, num_labels, threshold, average, **kwargs)
        raise ValueError(f"Task {task} not supported!")


class F1Score(_ClassificationTaskWrapper):
    """Task wrapper: returns Binary/Multiclass/MultilabelF1Score for ``task``."""

    def __new__(  # type: ignore[misc]
        cls: Type["F1Score"],
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
        kwargs.update({"multidim_average": multidim_average, "ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTask.BINARY:
            return BinaryF1Score(threshold, **kwargs)
        if task == ClassificationTask.MULTICLASS:
            if not isinstance(num_classes, int):
                raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
            if not isinstance(top_k, int):
                raise ValueError(f"`top_k` is expected to be `int` but `{type(top_k)} was passed.`")
            return MulticlassF1Score(num_classes, top_k, average, **kwargs)
        if task == ClassificationTask.MULTILABEL:
            if not isinstance(num_labels, int):
                raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
            return MultilabelF1Score(num_labels, threshold, average, **kwargs)
        raise ValueError(f"Task {task} not supported!")
