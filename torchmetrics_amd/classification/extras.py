"""Calibration error, hinge loss, label-ranking, exact match, group fairness and Dice module metrics.

Parity: reference ``S/classification/calibration_error.py``, ``hinge.py``, ``ranking.py``, ``exact_match.py``,
``group_fairness.py``, ``dice.py``.  State layouts (names, reductions) follow the reference so checkpoints and DDP
syncs are interchangeable.  Deliberate difference: ``BinaryGroupStatRates`` / ``BinaryFairness`` accumulate
statistics by group *id* (the reference enumerates the groups present in each batch, which misattributes counts when
a batch lacks a group).
"""
from typing import Any, Dict, Optional, Tuple, Type

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.classification.base import _ClassificationTaskWrapper
from torchmetrics_amd.functional.classification._legacy import _stat_scores_update
from torchmetrics_amd.functional.classification.calibration_error import _BOUNDARIES
from torchmetrics_amd.functional.classification.calibration_error import (
    _binary_calibration_error_arg_validation,
    _binary_float_preds_validation,
    _binary_format,
    _ce_compute,
    _multiclass_calibration_error_arg_validation,
    _multiclass_calibration_error_update,
    _multiclass_float_preds_validation,
    _multiclass_format,
)
from torchmetrics_amd.functional.classification.dice import _dice_compute
from torchmetrics_amd.functional.classification.exact_match import (
    _exact_match_fused,
    _exact_match_reduce,
    _multiclass_exact_match_format,
    _multiclass_exact_match_update,
    _multilabel_exact_match_format,
    _multilabel_exact_match_update,
)
from torchmetrics_amd.functional.classification.group_fairness import (
    _compute_binary_demographic_parity,
    _compute_binary_equal_opportunity,
    _group_stat_counts,
    _groups_validation,
)
from torchmetrics_amd.functional.classification.hinge import (
    _binary_hinge_loss_arg_validation,
    _binary_hinge_loss_update,
    _hinge_loss_compute,
    _multiclass_hinge_loss_arg_validation,
    _multiclass_hinge_loss_update,
)
from torchmetrics_amd.functional.classification.ranking import (
    _multilabel_coverage_error_update,
    _multilabel_ranking_arg_validation,
    _multilabel_ranking_average_precision_update,
    _multilabel_ranking_format,
    _multilabel_ranking_loss_update,
    _multilabel_ranking_tensor_validation,
    _ranking_reduce,
)
from torchmetrics_amd.functional.classification.stat_scores import (
    _binary_stat_scores_arg_validation,
    _binary_stat_scores_tensor_validation,
    _multiclass_stat_scores_arg_validation,
    _multiclass_stat_scores_tensor_validation,
    _multilabel_stat_scores_arg_validation,
    _multilabel_stat_scores_tensor_validation,
)
from torchmetrics_amd.functional.classification.stat_scores import _sink_flag
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.data import dim_zero_cat, dim_zero_sum
from torchmetrics_amd.utilities.enums import ClassificationTaskNoBinary, ClassificationTaskNoMultilabel
from torchmetrics_amd.utilities.prints import rank_zero_warn


# --------------------------------------------------------------------------------------------- calibration error
class _BinnedCalibration(Metric):
    """Incremental bins next to the reference's list states (``confidences`` / ``accuracies``, kept for API and
    state-dict parity).

    Every ROCm f32 update also adds its (count, Σconf, Σacc) bins into a per-metric ``[n_bins + 1, 3]`` cache (one
    launch), so ``compute()`` folds ``n_bins`` bins instead of re-binning every sample seen so far (the reference
    concatenates and bucketizes the whole history on each compute; with a compute per step that is O(steps²)).  The
    cache is trusted only while it covers exactly the samples in the list states (host-side element counts, no sync):
    anything else -- a forward() state merge, a loaded state dict, CPU states -- re-bins from the lists once and
    re-seeds the cache.

    Under DDP, ``sync()`` / ``sync_context`` gather the list states like the reference (``S/metric.py:427-457``: after
    a sync they are the global lists).  The sync that only serves ``compute()`` sends the bins instead: every rank
    offers its local ``[n_bins + 1, 3]`` bins (the cache, or one binning pass over its lists when the cache does not
    cover them) as an fp64 SUM state -- one bucket of the metric's / collection's single engine call, no agreement
    round, no host read -- and compute() folds the global bins."""

    _fold_cat_lists = True  # compute() only concatenates the list states
    _fold_every = 8  # (the bin cache serves compute(): the lists are folded every 8th batch, not at every compute)

    def _bounds(self, device: torch.device) -> Tensor:
        key = (self.n_bins, torch.float32, device)
        b = _BOUNDARIES.get(key)
        if b is None:
            b = _BOUNDARIES[key] = torch.linspace(0, 1, self.n_bins + 1, dtype=torch.float32, device=device)
        return b

    def _cache_add(self, conf: Tensor, acc: Tensor) -> None:
        if not (conf.is_cuda and conf.dtype == torch.float32 and self.n_bins + 1 <= 4096) or self.compute_on_cpu:
            self.__dict__.pop("_bin_cache", None)
            return
        cache = self.__dict__.get("_bin_cache")
        if cache is None or cache[0].device != conf.device or cache[2] is not self.confidences:
            if self._list_numel() != conf.numel():  # samples before this batch are not in any cache
                self.__dict__.pop("_bin_cache", None)
                return
            cache = [torch.zeros(self.n_bins + 1, 3, dtype=torch.float32, device=conf.device), 0, self.confidences]
            self.__dict__["_bin_cache"] = cache
        ops.calibration_bins_into(conf.contiguous(), acc.float().contiguous(), self._bounds(conf.device), cache[0])
        cache[1] += conf.numel()

    def _list_numel(self) -> int:
        c = self.confidences
        return c.numel() if isinstance(c, Tensor) else sum(x.numel() for x in c)

    def _valid_cache(self) -> Optional[list]:
        """The cache, if it covers exactly the samples in the list states: same list OBJECT (a loaded state dict,
        ``.to()`` or a forward merge rebinds the list) and the same element count."""
        cache = self.__dict__.get("_bin_cache")
        if cache is not None and cache[2] is self.confidences and cache[1] == self._list_numel() and cache[1] > 0:
            return cache
        if cache is not None:
            self.__dict__.pop("_bin_cache", None)  # drop it (and its reference to the replaced list)
        return None

    def reset(self) -> None:
        super().reset()
        self.__dict__.pop("_bin_cache", None)
        self.__dict__.pop("_bin_synced", None)

    def unsync(self, should_unsync: bool = True) -> None:
        # the globally reduced bins belong to the synced view only
        if should_unsync:
            self.__dict__.pop("_bin_synced", None)
        super().unsync(should_unsync)

    def _load_from_state_dict(self, *args: Any, **kwargs: Any) -> None:
        self.__dict__.pop("_bin_cache", None)
        super()._load_from_state_dict(*args, **kwargs)

    def _apply(self, fn: Any, exclude_state: Any = "") -> Any:
        self.__dict__.pop("_bin_cache", None)
        return super()._apply(fn, exclude_state)

    def _local_bins(self) -> Tensor:
        """This rank's (count, Σconf, Σacc) bins over every sample in its list states: the cache when it covers them,
        else one binning pass (re-seeding the cache on ROCm f32); always available, so every rank takes the same
        sync plan."""
        cache = self._valid_cache()
        if cache is not None:
            return cache[0]
        conf = dim_zero_cat(self.confidences) if self._list_numel() else None
        if conf is None:
            return torch.zeros(self.n_bins + 1, 3, dtype=torch.float64, device=self.device)
        acc = dim_zero_cat(self.accuracies)
        if conf.is_cuda and conf.dtype == torch.float32 and self.n_bins + 1 <= 4096 and not self.compute_on_cpu:
            cache = [torch.zeros(self.n_bins + 1, 3, dtype=torch.float32, device=conf.device), conf.numel(),
                     self.confidences]
            ops.calibration_bins_into(conf.contiguous(), acc.float().contiguous(), self._bounds(conf.device),
                                      cache[0])
            self.__dict__["_bin_cache"] = cache
            return cache[0]
        bounds = torch.linspace(0, 1, self.n_bins + 1, dtype=conf.dtype, device=conf.device)
        idx = torch.bucketize(conf, bounds, right=True) - 1
        src = torch.stack([torch.ones_like(conf), conf, acc.to(conf.dtype)], dim=1)
        return torch.zeros(self.n_bins + 1, 3, dtype=conf.dtype, device=conf.device).index_add_(0, idx, src)

    def _compute_sync_override(self) -> Optional[Tuple[Dict[str, Tensor], Dict[str, Any]]]:
        return {"bins\0": self._local_bins().to(torch.float64)}, {"bins\0": dim_zero_sum}

    def _compute_sync_finish(self, synced: Dict[str, Any]) -> None:
        c = self.confidences
        first = c if isinstance(c, Tensor) else (c[0] if c else None)
        # the global bins in the lists' dtype (the reference's compute runs in the confidences' dtype)
        dt = first.dtype if first is not None and first.is_floating_point() else torch.float32
        self.__dict__["_bin_synced"] = synced["bins\0"].to(torch.float32 if synced["bins\0"].is_cuda else dt)

    def compute(self) -> Tensor:
        bins = self.__dict__.pop("_bin_synced", None)
        if bins is None:
            cache = self._valid_cache()
            bins = cache[0] if cache is not None else None
        if bins is None:
            conf, acc = dim_zero_cat(self.confidences), dim_zero_cat(self.accuracies)
            if conf.is_cuda and conf.dtype == torch.float32 and not self._is_synced and self.n_bins + 1 <= 4096:
                # re-seed the cache from the lists (one binning pass, which this compute needs anyway)
                cache = [torch.zeros(self.n_bins + 1, 3, dtype=torch.float32, device=conf.device), 0,
                         self.confidences]
                ops.calibration_bins_into(conf.contiguous(), acc.float().contiguous(), self._bounds(conf.device),
                                          cache[0])
                cache[1] = conf.numel()
                self.__dict__["_bin_cache"] = cache
                bins = cache[0]
            else:
                return _ce_compute(conf, acc, self.n_bins, norm=self.norm)
        if self.norm in ("l1", "max") and bins.is_cuda:
            return ops.calibration_error_from_bins(bins, self.norm)
        count = bins[:, 0]
        if self.norm in ("l1", "max"):
            acc_bin = torch.nan_to_num(bins[:, 2] / count)
            conf_bin = torch.nan_to_num(bins[:, 1] / count)
            if self.norm == "l1":
                return torch.sum(torch.abs(acc_bin - conf_bin) * (count / count.sum()))
            return torch.max(torch.abs(acc_bin - conf_bin))
        acc_bin = torch.nan_to_num(bins[:, 2] / count)
        conf_bin = torch.nan_to_num(bins[:, 1] / count)
        ce = torch.sum(torch.pow(acc_bin - conf_bin, 2) * (count / count.sum()))
        return torch.where(ce > 0, ce.sqrt(), torch.zeros_like(ce))


class BinaryCalibrationError(_BinnedCalibration):
    """Top-label calibration error (ECE / MCE / RMSCE) for binary probabilities."""

    is_differentiable: bool = False
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, n_bins: int = 15, norm: Literal["l1", "l2", "max"] = "l1", ignore_index: Optional[int] = None,
                 validate_args: bool = True, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _binary_calibration_error_arg_validation(n_bins, norm, ignore_index)
        self.validate_args = validate_args
        self.n_bins = n_bins
        self.norm = norm
        self.ignore_index = ignore_index
        self.add_state("confidences", [], dist_reduce_fx="cat")
        self.add_state("accuracies", [], dist_reduce_fx="cat")

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _binary_float_preds_validation(preds, target, self.ignore_index)
        preds, target = _binary_format(preds, target, self.ignore_index)
        self.confidences.append(preds)
        self.accuracies.append(target)
        self._cache_add(preds, target)


class MulticlassCalibrationError(_BinnedCalibration):
    """Top-label calibration error for multiclass probabilities / logits."""

    is_differentiable: bool = False
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def __init__(self, num_classes: int, n_bins: int = 15, norm: Literal["l1", "l2", "max"] = "l1",
                 ignore_index: Optional[int] = None, validate_args: bool = True, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multiclass_calibration_error_arg_validation(num_classes, n_bins, norm, ignore_index)
        self.validate_args = validate_args
        self.num_classes = num_classes
        self.n_bins = n_bins
        self.norm = norm
        self.ignore_index = ignore_index
        self.add_state("confidences", [], dist_reduce_fx="cat")
        self.add_state("accuracies", [], dist_reduce_fx="cat")

    def update(self, preds: Tensor, target: Tensor) -> None:
        if (preds.is_cuda and self.ignore_index is None and preds.ndim == 2 and target.ndim == 1
                and preds.dtype in (torch.float32, torch.float16, torch.bfloat16) and not target.is_floating_point()):
            # fused path: validation range bits, softmax-or-not decision, top-1 and correctness in two launches
            flag = None
            if self.validate_args:
                _multiclass_float_preds_validation(preds, target, self.num_classes, None, check_values=False)
                flag = self._device_error_buffer(preds.device)
            ws = self.__dict__.get("_calib_ws")
            if ws is None:
                ws = self.__dict__["_calib_ws"] = ops.CalibrationWorkspace()
            confidences, accuracies = ops.mc_calibration_update(preds, target, ws, flag)
            self.confidences.append(confidences)
            self.accuracies.append(accuracies)
            self._cache_add(confidences, accuracies)
            return
        if self.validate_args:
            flag = self._device_error_buffer(preds.device) if preds.is_cuda else None
            _multiclass_float_preds_validation(preds, target, self.num_classes, self.ignore_index, flag)
        preds, target = _multiclass_format(preds, target, self.ignore_index)
        confidences, accuracies = _multiclass_calibration_error_update(preds, target)
        self.confidences.append(confidences)
        self.accuracies.append(accuracies)
        self._cache_add(confidences, accuracies)


class CalibrationError(_ClassificationTaskWrapper):
    """Task wrapper for the calibration error."""

    def __new__(cls: Type["CalibrationError"], task: Literal["binary", "multiclass"], n_bins: int = 15,
                norm: Literal["l1", "l2", "max"] = "l1", num_classes: Optional[int] = None,
                ignore_index: Optional[int] = None, validate_args: bool = True, **kwargs: Any) -> Metric:
        task = ClassificationTaskNoMultilabel.from_str(task)
        kwargs.update({"n_bins": n_bins, "norm": norm, "ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTaskNoMultilabel.BINARY:
            return BinaryCalibrationError(**kwargs)
        if task == ClassificationTaskNoMultilabel.MULTICLASS:
            if not isinstance(num_classes, int):
                raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
            return MulticlassCalibrationError(num_classes, **kwargs)
        raise ValueError(f"Not handled value: {task}")


# ---------------------------------------------------------------------------------------------------- hinge loss
class BinaryHingeLoss(Metric):
    """Mean (squared) hinge loss for binary tasks."""

    is_differentiable: bool = True
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, squared: bool = False, ignore_index: Optional[int] = None, validate_args: bool = True,
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _binary_hinge_loss_arg_validation(squared, ignore_index)
        self.validate_args = validate_args
        self.squared = squared
        self.ignore_index = ignore_index
        self.add_state("measures", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", default=torch.tensor(0), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        if _hinge_fusable(self, preds, target):
            # one pass + one fold on the device; target values are checked by the kernel (raised at compute)
            if self.validate_args:
                _check_same_shape(preds, target)
            ops.hinge_update(preds.reshape(-1).contiguous(), target.reshape(-1).contiguous(), ops.HINGE_BINARY,
                             self.squared, self.ignore_index, self.__dict__, self.measures, self.total,
                             self._hinge_flag(preds))
            return
        if self.validate_args:
            _binary_float_preds_validation(preds, target, self.ignore_index)
        measures, total = _binary_hinge_loss_update(preds, target, self.squared, self.ignore_index)
        self.measures += measures
        self.total += total

    def _hinge_flag(self, preds: Tensor) -> Tensor:
        return self._device_error_buffer(preds.device) if self.validate_args else _sink_flag(preds.device)

    def compute(self) -> Tensor:
        return _hinge_loss_compute(self.measures, self.total)


def _hinge_fusable(m: Metric, preds: Tensor, target: Tensor) -> bool:
    """ROCm float scores, integer targets, in-place-updatable states and no gradient to track."""
    st, tot = m.measures, m.total
    return (preds.is_cuda and preds.is_floating_point() and not target.is_floating_point()
            and preds.dtype in (torch.float32, torch.float16, torch.bfloat16, torch.float64)
            and target.dtype in (torch.int64, torch.int32, torch.uint8, torch.bool)
            and isinstance(st, Tensor) and st.device == preds.device and st.dtype in (torch.float32, torch.float64)
            and st.is_contiguous() and isinstance(tot, Tensor) and tot.device == preds.device
            and tot.dtype == torch.int64 and tot.numel() == 1
            and preds.numel() > 0
            and not (torch.is_grad_enabled() and preds.requires_grad))


class MulticlassHingeLoss(Metric):
    """Mean (squared) multiclass hinge loss (Crammer-Singer or one-vs-all)."""

    is_differentiable: bool = True
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def __init__(self, num_classes: int, squared: bool = False,
                 multiclass_mode: Literal["crammer-singer", "one-vs-all"] = "crammer-singer",
                 ignore_index: Optional[int] = None, validate_args: bool = True, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multiclass_hinge_loss_arg_validation(num_classes, squared, multiclass_mode, ignore_index)
        self.validate_args = validate_args
        self.num_classes = num_classes
        self.squared = squared
        self.multiclass_mode = multiclass_mode
        self.ignore_index = ignore_index
        self.add_state(
            "measures",
            default=torch.tensor(0.0) if multiclass_mode == "crammer-singer" else torch.zeros(num_classes),
            dist_reduce_fx="sum",
        )
        self.add_state("total", default=torch.tensor(0), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        if _hinge_fusable(self, preds, target):
            flag = self._device_error_buffer(preds.device) if self.validate_args else _sink_flag(preds.device)
            if self.validate_args:
                _multiclass_float_preds_validation(preds, target, self.num_classes, self.ignore_index, flag,
                                                   check_values=False)
            c = preds.shape[1]
            rows = preds.movedim(1, -1).reshape(-1, c).contiguous()
            mode = ops.HINGE_CRAMMER_SINGER if self.multiclass_mode == "crammer-singer" else ops.HINGE_ONE_VS_ALL
            ops.hinge_update(rows, target.reshape(-1).contiguous(), mode, self.squared, self.ignore_index,
                             self.__dict__, self.measures, self.total, flag)
            return
        if self.validate_args:
            _multiclass_float_preds_validation(preds, target, self.num_classes, self.ignore_index)
        measures, total = _multiclass_hinge_loss_update(preds, target, self.squared, self.multiclass_mode,
                                                        self.ignore_index)
        self.measures += measures
        self.total += total

    def compute(self) -> Tensor:
        return _hinge_loss_compute(self.measures, self.total)


class HingeLoss(_ClassificationTaskWrapper):
    """Task wrapper for the hinge loss."""

    def __new__(cls: Type["HingeLoss"], task: Literal["binary", "multiclass"], num_classes: Optional[int] = None,
                squared: bool = False, multiclass_mode: Optional[Literal["crammer-singer", "one-vs-all"]] = "crammer-singer",
                ignore_index: Optional[int] = None, validate_args: bool = True, **kwargs: Any) -> Metric:
        task = ClassificationTaskNoMultilabel.from_str(task)
        kwargs.update({"ignore_index": ignore_index, "validate_args": validate_args})
        if task == ClassificationTaskNoMultilabel.BINARY:
            return BinaryHingeLoss(squared, **kwargs)
        if task == ClassificationTaskNoMultilabel.MULTICLASS:
            if not isinstance(num_classes, int):
                raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
            return MulticlassHingeLoss(num_classes, squared, multiclass_mode, **kwargs)
        raise ValueError(f"Unsupported task `{task}`")


# ------------------------------------------------------------------------------------------------ label ranking
class _RankingBase(Metric):
    is_differentiable: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Label"
    _update_fn: Any = None

    def __init__(self, num_labels: int, ignore_index: Optional[int] = None, validate_args: bool = True,
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multilabel_ranking_arg_validation(num_labels, ignore_index)
        self.validate_args = validate_args
        self.num_labels = num_labels
        self.ignore_index = ignore_index
        self.add_state("measure", torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", torch.tensor(0.0), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _multilabel_ranking_tensor_validation(preds, target, self.num_labels, self.ignore_index)
        preds, target = _multilabel_ranking_format(preds, target, self.num_labels, self.ignore_index)
        measure, num_elements = type(self)._update_fn(preds, target)
        self.measure += measure
        self.total += num_elements

    def compute(self) -> Tensor:
        return _ranking_reduce(self.measure, self.total)


class MultilabelCoverageError(_RankingBase):
    """Average depth into the ranked labels needed to cover all relevant labels."""

    higher_is_better: bool = False
    _update_fn = staticmethod(_multilabel_coverage_error_update)


class MultilabelRankingAveragePrecision(_RankingBase):
    """Label ranking average precision (LRAP)."""

    higher_is_better: bool = True
    _update_fn = staticmethod(_multilabel_ranking_average_precision_update)


class MultilabelRankingLoss(_RankingBase):
    """Label ranking loss (fraction of mis-ordered relevant/irrelevant pairs)."""

    higher_is_better: bool = False
    _update_fn = staticmethod(_multilabel_ranking_loss_update)


# -------------------------------------------------------------------------------------------------- exact match
class _ExactMatchBase(Metric):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def _create_states(self) -> None:
        samplewise = self.multidim_average == "samplewise"
        self.add_state("correct", [] if samplewise else torch.zeros(1, dtype=torch.long),
                       dist_reduce_fx="cat" if samplewise else "sum")
        self.add_state("total", torch.zeros(1, dtype=torch.long), dist_reduce_fx="mean" if samplewise else "sum")

    def _accumulate(self, correct: Tensor, total: Tensor) -> None:
        if self.multidim_average == "samplewise":
            self.correct.append(correct)
            self.total = total
        else:
            self.correct += correct
            self.total += total

    def _fused(self, preds: Tensor, target: Tensor, multilabel: bool, num: int, threshold: float) -> bool:
        """ROCm: one exact-match kernel pass; global states are updated in place (no per-batch temporaries)."""
        if self.multidim_average == "samplewise":
            out = _exact_match_fused(preds, target, multilabel, num, threshold, "samplewise", self.ignore_index,
                                     self.__dict__)
            if out is None:
                return False
            self._accumulate(*out)
            return True
        correct, total = self.correct, self.total
        if not (isinstance(correct, Tensor) and correct.is_cuda and correct.dtype == torch.int64 and total.is_cuda):
            return False
        return _exact_match_fused(preds, target, multilabel, num, threshold, "global", self.ignore_index,
                                  self.__dict__, correct, total) is not None

    def compute(self) -> Tensor:
        correct = dim_zero_cat(self.correct) if isinstance(self.correct, list) else self.correct
        return _exact_match_reduce(correct, self.total)


class MulticlassExactMatch(_ExactMatchBase):
    """Exact match for multi-dimensional multiclass inputs (all positions of a sample correct)."""

    plot_legend_name: str = "Class"

    def __init__(self, num_classes: int, multidim_average: Literal["global", "samplewise"] = "global",
                 ignore_index: Optional[int] = None, validate_args: bool = True, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multiclass_stat_scores_arg_validation(num_classes, 1, None, multidim_average, ignore_index)
        self.num_classes = num_classes
        self.multidim_average = multidim_average
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_states()

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _multiclass_stat_scores_tensor_validation(preds, target, self.num_classes, self.multidim_average,
                                                      self.ignore_index)
        if self._fused(preds, target, False, self.num_classes, 0.5):
            return
        preds, target = _multiclass_exact_match_format(preds, target)
        self._accumulate(*_multiclass_exact_match_update(preds, target, self.multidim_average, self.ignore_index))


class MultilabelExactMatch(_ExactMatchBase):
    """Exact match for multilabel inputs (the whole label set of a sample correct)."""

    plot_legend_name: str = "Label"

    def __init__(self, num_labels: int, threshold: float = 0.5,
                 multidim_average: Literal["global", "samplewise"] = "global", ignore_index: Optional[int] = None,
                 validate_args: bool = True, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _multilabel_stat_scores_arg_validation(num_labels, threshold, None, multidim_average, ignore_index)
        self.num_labels = num_labels
        self.threshold = threshold
        self.multidim_average = multidim_average
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_states()

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.validate_args:
            _multilabel_stat_scores_tensor_validation(preds, target, self.num_labels, self.multidim_average,
                                                      self.ignore_index)
        if self._fused(preds, target, True, self.num_labels, self.threshold):
            return
        preds, target = _multilabel_exact_match_format(preds, target, self.num_labels, self.threshold,
                                                       self.ignore_index)
        self._accumulate(*_multilabel_exact_match_update(preds, target, self.num_labels, self.multidim_average))


class ExactMatch(_ClassificationTaskWrapper):
    """Task wrapper for exact match."""

    def __new__(cls: Type["ExactMatch"], task: Literal["binary", "multiclass", "multilabel"], threshold: float = 0.5,
                num_classes: Optional[int] = None, num_labels: Optional[int] = None,
                multidim_average: Literal["global", "samplewise"] = "global", ignore_index: Optional[int] = None,
                validate_args: bool = True, **kwargs: Any) -> Metric:
        task = ClassificationTaskNoBinary.from_str(task)
        kwargs.update({"multidim_average": multidim_average, "ignore_index": ignore_index,
                       "validate_args": validate_args})
        if task == ClassificationTaskNoBinary.MULTICLASS:
            if not isinstance(num_classes, int):
                raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
            return MulticlassExactMatch(num_classes, **kwargs)
        if task == ClassificationTaskNoBinary.MULTILABEL:
            if not isinstance(num_labels, int):
                raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
            return MultilabelExactMatch(num_labels, threshold, **kwargs)
        raise ValueError(f"Task {task} not supported!")


# ---------------------------------------------------------------------------------------------- group fairness
class _AbstractGroupStatScores(Metric):
    tp: Tensor
    fp: Tensor
    tn: Tensor
    fn: Tensor

    def _create_states(self, num_groups: int) -> None:
        for s in ("tp", "fp", "tn", "fn"):
            self.add_state(s, torch.zeros(num_groups, dtype=torch.long), dist_reduce_fx="sum")

    def _group_update(self, preds: Tensor, target: Tensor, groups: Tensor) -> None:
        if self.validate_args:
            _binary_stat_scores_tensor_validation(preds, target, "global", self.ignore_index)
            _groups_validation(groups, self.num_groups)
        states = (self.tp, self.fp, self.tn, self.fn)
        if (preds.is_cuda and all(isinstance(t, Tensor) and t.device == preds.device and t.dtype == torch.int64
                                  for t in states) and target.device == preds.device
                and groups.device == preds.device and preds.numel() == target.numel() == groups.numel()):
            ops.group_stats_update(preds, target, groups, self.num_groups, self.threshold, self.ignore_index,
                                   self.__dict__, *states)
            return
        counts = _group_stat_counts(preds, target, groups, self.num_groups, self.threshold, self.ignore_index)
        self.tp += counts[:, 0]
        self.fp += counts[:, 1]
        self.tn += counts[:, 2]
        self.fn += counts[:, 3]


class BinaryGroupStatRates(_AbstractGroupStatScores):
    """tp/fp/tn/fn rates per group for binary predictions."""

    is_differentiable: bool = False
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, num_groups: int, threshold: float = 0.5, ignore_index: Optional[int] = None,
                 validate_args: bool = True, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _binary_stat_scores_arg_validation(threshold, "global", ignore_index)
        if not isinstance(num_groups, int) and num_groups < 2:
            raise ValueError(f"Expected argument `num_groups` to be an int larger than 1, but got {num_groups}")
        self.num_groups = num_groups
        self.threshold = threshold
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_states(num_groups)

    def update(self, preds: Tensor, target: Tensor, groups: Tensor) -> None:
        self._group_update(preds, target, groups)

    def compute(self) -> Dict[str, Tensor]:
        results = torch.stack((self.tp, self.fp, self.tn, self.fn), dim=1)
        return {f"group_{i}": group / group.sum() for i, group in enumerate(results)}


class BinaryFairness(_AbstractGroupStatScores):
    """Demographic parity and/or equal opportunity across groups."""

    is_differentiable: bool = False
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, num_groups: int,
                 task: Literal["demographic_parity", "equal_opportunity", "all"] = "all", threshold: float = 0.5,
                 ignore_index: Optional[int] = None, validate_args: bool = True, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if task not in ["demographic_parity", "equal_opportunity", "all"]:
            raise ValueError(
                f"Expected argument `task` to either be ``demographic_parity``,"
                f"``equal_opportunity`` or ``all`` but got {task}."
            )
        if validate_args:
            _binary_stat_scores_arg_validation(threshold, "global", ignore_index)
        if not isinstance(num_groups, int) and num_groups < 2:
            raise ValueError(f"Expected argument `num_groups` to be an int larger than 1, but got {num_groups}")
        self.num_groups = num_groups
        self.task = task
        self.threshold = threshold
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_states(num_groups)

    def update(self, preds: Tensor, target: Tensor, groups: Tensor) -> None:
        if self.task == "demographic_parity":
            if target is not None:
                rank_zero_warn("The task demographic_parity does not require a target.", UserWarning)
            target = torch.zeros(preds.shape, dtype=torch.long, device=preds.device)
        self._group_update(preds, target, groups)

    def compute(self) -> Dict[str, Tensor]:
        st = (self.tp, self.fp, self.tn, self.fn)
        if self.task == "demographic_parity":
            return _compute_binary_demographic_parity(*st)
        if self.task == "equal_opportunity":
            return _compute_binary_equal_opportunity(*st)
        return {**_compute_binary_demographic_parity(*st), **_compute_binary_equal_opportunity(*st)}


# ---------------------------------------------------------------------------------------------------------- Dice
class Dice(Metric):
    """Dice score with the legacy task-less input API."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    plot_legend_name: str = "Class"

    def __init__(self, zero_division: int = 0, num_classes: Optional[int] = None, threshold: float = 0.5,
                 average: Optional[Literal["micro", "macro", "none"]] = "micro", mdmc_average: Optional[str] = "global",
                 ignore_index: Optional[int] = None, top_k: Optional[int] = None, multiclass: Optional[bool] = None,
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        allowed_average = ("micro", "macro", "samples", "none", None)
        if average not in allowed_average:
            raise ValueError(f"The `average` has to be one of {allowed_average}, got {average}.")
        self.reduce = average
        self.mdmc_reduce = mdmc_average
        self.num_classes = num_classes
        self.threshold = threshold
        self.multiclass = multiclass
        self.ignore_index = ignore_index
        self.top_k = top_k
        if average not in ["micro", "macro", "samples"]:
            raise ValueError(f"The `reduce` {average} is not valid.")
        if mdmc_average not in [None, "samplewise", "global"]:
            raise ValueError(f"The `mdmc_reduce` {mdmc_average} is not valid.")
        if average == "macro" and (not num_classes or num_classes < 1):
            raise ValueError("When you set `average` as 'macro', you have to provide the number of classes.")
        if num_classes and ignore_index is not None and (not ignore_index < num_classes or num_classes == 1):
            raise ValueError(f"The `ignore_index` {ignore_index} is not valid for inputs with {num_classes} classes")
        listed = mdmc_average == "samplewise" or average == "samples"
        for s in ("tp", "fp", "tn", "fn"):
            default = [] if listed else torch.zeros([] if average == "micro" else [num_classes], dtype=torch.long)
            self.add_state(s, default=default, dist_reduce_fx="cat" if listed else "sum")
        self.average = average
        self.zero_division = zero_division

    def update(self, preds: Tensor, target: Tensor) -> None:
        tp, fp, tn, fn = _stat_scores_update(
            preds, target, reduce=self.reduce, mdmc_reduce=self.mdmc_reduce, threshold=self.threshold,
            num_classes=self.num_classes, top_k=self.top_k, multiclass=self.multiclass,
            ignore_index=self.ignore_index,
        )
        if isinstance(self.tp, list):
            self.tp.append(tp)
            self.fp.append(fp)
            self.tn.append(tn)
            self.fn.append(fn)
        else:
            self.tp += tp
            self.fp += fp
            self.tn += tn
            self.fn += fn

    def compute(self) -> Tensor:
        cat = lambda x: torch.cat(x) if isinstance(x, list) else x  # noqa: E731
        return _dice_compute(cat(self.tp), cat(self.fp), cat(self.fn), self.average, self.mdmc_reduce,
                             self.zero_division)
