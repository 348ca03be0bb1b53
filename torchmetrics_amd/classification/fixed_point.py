"""Operating-point module metrics on top of the curve states.

Parity: reference ``S/classification/recall_fixed_precision.py``, ``precision_fixed_recall.py``,
``sensitivity_specificity.py``, ``specificity_sensitivity.py``.  Each class shares the binned / unbinned curve state
of :mod:`~torchmetrics_amd.classification.precision_recall_curve` and returns ``(value, threshold)``.
"""
import inspect
from typing import Any, Optional, Tuple, Type

from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_amd.classification.precision_recall_curve import (
    BinaryPrecisionRecallCurve,
    MulticlassPrecisionRecallCurve,
    MultilabelPrecisionRecallCurve,
    _curve_task,
)
from torchmetrics_amd.functional.classification.precision_recall_curve import Thresholds
from torchmetrics_amd.functional.classification.recall_fixed_precision import (
    _KIND_CURVE,
    _binary_precision_recall_curve_arg_validation,
    _check_min,
    _fixed_compute,
    _multiclass_precision_recall_curve_arg_validation,
    _multilabel_precision_recall_curve_arg_validation,
    _pr_reduce,
)
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class _FixedMixin:
    _kind: str
    _min_name: str
    higher_is_better: Optional[bool] = None
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def _fixed(self, task: str, num: int = 0, ignore_index: Optional[int] = None) -> Tuple[Tensor, Tensor]:
        return _fixed_compute(_KIND_CURVE[self._kind], task, _pr_reduce(self._kind), self._state(), self.thresholds,
                              getattr(self, self._min_name), num, ignore_index)

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        val = val or self.compute()[0]
        return self._plot(val, ax)


def _make(kind: str, min_name: str, prefix: str):
    class _Binary(_FixedMixin, BinaryPrecisionRecallCurve):
        _kind = kind
        _min_name = min_name

        def __init__(self, min_value: float, thresholds: Thresholds = None, ignore_index: Optional[int] = None,
                     validate_args: bool = True, **kwargs: Any) -> None:
            super().__init__(thresholds=thresholds, ignore_index=ignore_index, validate_args=False, **kwargs)
            if validate_args:
                _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
                _check_min(min_name, min_value)
            self.validate_args = validate_args
            setattr(self, min_name, min_value)

        def compute(self) -> Tuple[Tensor, Tensor]:
            return self._fixed("binary")

    class _Multiclass(_FixedMixin, MulticlassPrecisionRecallCurve):
        _kind = kind
        _min_name = min_name
        plot_legend_name: str = "Class"

        def __init__(self, num_classes: int, min_value: float, thresholds: Thresholds = None,
                     ignore_index: Optional[int] = None, validate_args: bool = True, **kwargs: Any) -> None:
            super().__init__(num_classes=num_classes, thresholds=thresholds, ignore_index=ignore_index,
                             validate_args=False, **kwargs)
            if validate_args:
                _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index)
                _check_min(min_name, min_value)
            self.validate_args = validate_args
            setattr(self, min_name, min_value)

        def compute(self) -> Tuple[Tensor, Tensor]:
            return self._fixed("multiclass", self.num_classes)

    class _Multilabel(_FixedMixin, MultilabelPrecisionRecallCurve):
        _kind = kind
        _min_name = min_name
        plot_legend_name: str = "Label"

        def __init__(self, num_labels: int, min_value: float, thresholds: Thresholds = None,
                     ignore_index: Optional[int] = None, validate_args: bool = True, **kwargs: Any) -> None:
            super().__init__(num_labels=num_labels, thresholds=thresholds, ignore_index=ignore_index,
                             validate_args=False, **kwargs)
            if validate_args:
                _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
                _check_min(min_name, min_value)
            self.validate_args = validate_args
            setattr(self, min_name, min_value)

        def compute(self) -> Tuple[Tensor, Tensor]:
            return self._fixed("multilabel", self.num_labels, self.ignore_index)

    for cls, task in ((_Binary, "Binary"), (_Multiclass, "Multiclass"), (_Multilabel, "Multilabel")):
        cls.__name__ = cls.__qualname__ = f"{task}{prefix}"
        cls.__doc__ = f"{task} {kind.replace('@', ' at fixed ')} (returns value and threshold)."
    return _Binary, _Multiclass, _Multilabel


def _named_init(cls, min_name: str, positional_num: Optional[str]):
    """Give the generated ``__init__`` the reference keyword name for the constraint (``min_precision`` ...)."""
    base_init = cls.__init__

    if positional_num is None:
        def __init__(self, *args: Any, **kwargs: Any) -> None:
            if min_name in kwargs:
                kwargs["min_value"] = kwargs.pop(min_name)
            base_init(self, *args, **kwargs)
    else:
        def __init__(self, *args: Any, **kwargs: Any) -> None:
            if positional_num in kwargs:
                kwargs["num_classes" if positional_num == "num_classes" else "num_labels"] = kwargs.pop(positional_num)
            if min_name in kwargs:
                kwargs["min_value"] = kwargs.pop(min_name)
            base_init(self, *args, **kwargs)
    # introspection shows the reference signature (``min_precision`` ... in its reference position)
    params = [inspect.Parameter("self", inspect.Parameter.POSITIONAL_OR_KEYWORD)]
    if positional_num is not None:
        params.append(inspect.Parameter(positional_num, inspect.Parameter.POSITIONAL_OR_KEYWORD))
    params += [inspect.Parameter(min_name, inspect.Parameter.POSITIONAL_OR_KEYWORD),
               inspect.Parameter("thresholds", inspect.Parameter.POSITIONAL_OR_KEYWORD, default=None),
               inspect.Parameter("ignore_index", inspect.Parameter.POSITIONAL_OR_KEYWORD, default=None),
               inspect.Parameter("validate_args", inspect.Parameter.POSITIONAL_OR_KEYWORD, default=True),
               inspect.Parameter("kwargs", inspect.Parameter.VAR_KEYWORD)]
    __init__.__signature__ = inspect.Signature(params)
    cls.__init__ = __init__
    return cls


def _family(kind: str, min_name: str, prefix: str):
    b, mc, ml = _make(kind, min_name, prefix)
    return _named_init(b, min_name, None), _named_init(mc, min_name, "num_classes"), _named_init(ml, min_name,
                                                                                                 "num_labels")


BinaryRecallAtFixedPrecision, MulticlassRecallAtFixedPrecision, MultilabelRecallAtFixedPrecision = _family(
    "recall@precision", "min_precision", "RecallAtFixedPrecision")
BinaryPrecisionAtFixedRecall, MulticlassPrecisionAtFixedRecall, MultilabelPrecisionAtFixedRecall = _family(
    "precision@recall", "min_recall", "PrecisionAtFixedRecall")
BinarySensitivityAtSpecificity, MulticlassSensitivityAtSpecificity, MultilabelSensitivityAtSpecificity = _family(
    "sensitivity@specificity", "min_specificity", "SensitivityAtSpecificity")
BinarySpecificityAtSensitivity, MulticlassSpecificityAtSensitivity, MultilabelSpecificityAtSensitivity = _family(
    "specificity@sensitivity", "min_sensitivity", "SpecificityAtSensitivity")


def _wrapper(name: str, min_name: str, classes):
    # reference order: (task, <min_name>, thresholds, num_classes, num_labels, ignore_index, validate_args)
    order = (min_name, "thresholds", "num_classes", "num_labels", "ignore_index", "validate_args")
    defaults = {"thresholds": None, "num_classes": None, "num_labels": None, "ignore_index": None,
                "validate_args": True}

    def __new__(cls: Type, task: Literal["binary", "multiclass", "multilabel"], *args: Any, **kwargs: Any) -> Metric:
        if len(args) > len(order):
            raise TypeError(f"{name}() takes at most {len(order) + 1} positional arguments")
        for key, val in zip(order, args):
            if key in kwargs:
                raise TypeError(f"{name}() got multiple values for argument '{key}'")
            kwargs[key] = val
        if min_name not in kwargs:
            raise TypeError(f"{name}() missing required argument: '{min_name}'")
        min_value = kwargs.pop(min_name)
        opts = {k: kwargs.pop(k, d) for k, d in defaults.items()}
        kwargs.update({"thresholds": opts["thresholds"], "ignore_index": opts["ignore_index"],
                       "validate_args": opts["validate_args"]})
        return _curve_task(*classes, task, opts["num_classes"], opts["num_labels"], kwargs,
                           bin_extra={"min_value": min_value}, mc_extra={"min_value": min_value},
                           ml_extra={"min_value": min_value})

    __new__.__signature__ = inspect.Signature(
        [inspect.Parameter("cls", inspect.Parameter.POSITIONAL_OR_KEYWORD),
         inspect.Parameter("task", inspect.Parameter.POSITIONAL_OR_KEYWORD),
         inspect.Parameter(min_name, inspect.Parameter.POSITIONAL_OR_KEYWORD)]
        + [inspect.Parameter(k, inspect.Parameter.POSITIONAL_OR_KEYWORD, default=defaults[k]) for k in order[1:]]
        + [inspect.Parameter("kwargs", inspect.Parameter.VAR_KEYWORD)])
    return type(name, (_ClassificationTaskWrapper,), {"__new__": __new__, "__doc__": f"Task wrapper for {name}."})


RecallAtFixedPrecision = _wrapper(
    "RecallAtFixedPrecision", "min_precision",
    (BinaryRecallAtFixedPrecision, MulticlassRecallAtFixedPrecision, MultilabelRecallAtFixedPrecision))
PrecisionAtFixedRecall = _wrapper(
    "PrecisionAtFixedRecall", "min_recall",
    (BinaryPrecisionAtFixedRecall, MulticlassPrecisionAtFixedRecall, MultilabelPrecisionAtFixedRecall))
SensitivityAtSpecificity = _wrapper(
    "SensitivityAtSpecificity", "min_specificity",
    (BinarySensitivityAtSpecificity, MulticlassSensitivityAtSpecificity, MultilabelSensitivityAtSpecificity))
SpecificityAtSensitivity = _wrapper(
    "SpecificityAtSensitivity", "min_sensitivity",
    (BinarySpecificityAtSensitivity, MulticlassSpecificityAtSensitivity, MultilabelSpecificityAtSensitivity))
