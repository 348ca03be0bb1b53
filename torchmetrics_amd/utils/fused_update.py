"""One fused update for a :class:`~torchmetrics_amd.MetricCollection`'s few-class multiclass members (SURVEY.md
section 7.1.3: "a collection's compute group runs ONE kernel per step").

The reference updates every compute group's leader separately (``S/collections.py:200-226``) and each leader re-reads
the batch.  Here, when a collection update hands the same ``(preds [N, C] logits / probabilities, target [N])`` to
leaders of the families below, they are served by ``ops.mc_family_update``
(``csrc/classification/family.hip``): ONE pass over the batch plus one fold launch, whatever the number of members:

* the stat-score family (``MulticlassStatScores`` and its Accuracy / Precision / Recall / F-beta / Specificity /
  Hamming subclasses) with ``top_k=1``, ``multidim_average="global"``;
* the confusion-matrix family (``MulticlassConfusionMatrix`` and its Jaccard / Cohen kappa / Matthews subclasses);
* the binned multiclass PR-curve family (PR curve / ROC / AUROC / average precision with tensor thresholds, one
  threshold set per launch; PR curve / ROC not ``average="micro"``; AUROC / AP keep per-class curve states whatever
  their ``average``);
* ``MulticlassCalibrationError``.

Every member must have ``ignore_index=None``, ``num_classes = C <= 64`` and the class's own ``update`` (a subclass
overriding it keeps its own).  Anything else -- CPU tensors, other shapes or dtypes, gradients, ``compute_on_cpu``,
states moved or replaced -- takes the members' own updates, which raise the reference's errors.  The fused update
does what each member's update does: the states accumulate in place, list states get their new elements, the
validation words get the device-side target-range bit, and ``_update_count`` / ``_computed`` are maintained.
"""
import operator
from typing import Any, Dict, List, Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_amd import ops

_MAX_C = 64
_MAX_CONS = 4
_LDS_WORDS = 15000  # the rows kernel's per-block image must fit in 64 KiB of LDS (with thresholds and bounds)


def _classes() -> Dict[str, type]:
    from torchmetrics_amd.classification.confusion_matrix import MulticlassConfusionMatrix
    from torchmetrics_amd.classification.extras import MulticlassCalibrationError
    from torchmetrics_amd.classification.precision_recall_curve import MulticlassPrecisionRecallCurve
    from torchmetrics_amd.classification.stat_scores import MulticlassStatScores

    return {"st": MulticlassStatScores, "cm": MulticlassConfusionMatrix, "cv": MulticlassPrecisionRecallCurve,
            "cb": MulticlassCalibrationError}


def _curve_wrappers() -> tuple:
    from torchmetrics_amd.classification.precision_recall_curve import MulticlassAUROC, MulticlassAveragePrecision

    return (MulticlassAUROC.update, MulticlassAveragePrecision.update)


def _role(m: Any) -> Optional[str]:
    """The family a metric joins the fused update as, or None."""
    cls = _classes()
    d = m.__dict__
    if d.get("compute_on_cpu") or d.get("ignore_index") is not None:
        return None
    c = d.get("num_classes")
    if not isinstance(c, int) or not 1 <= c <= _MAX_C:
        return None
    t = type(m)
    if isinstance(m, cls["st"]) and t.update is cls["st"].update:
        if d.get("top_k") == 1 and d.get("multidim_average") == "global":
            return "st"
        return None
    if isinstance(m, cls["cm"]) and t.update is cls["cm"].update:
        return "cm"
    if isinstance(m, cls["cv"]) and (t.update is cls["cv"].update or t.update in _curve_wrappers()):
        # AUROC / AP wrap the curve update with a transient average=None (their curve state is always per class)
        per_class = t.update is not cls["cv"].update or d.get("average") != "micro"
        if per_class and isinstance(d.get("_buffers", {}).get("thresholds"), Tensor):
            return "cv"
        return None
    if isinstance(m, cls["cb"]) and t.update is cls["cb"].update:
        return "cb"
    return None


class FamilyPlan:
    """The fusable members of one collection update (recorded once, re-checked per call by identity tests)."""

    def __init__(self, members: List[Tuple[str, Any]]) -> None:
        roles: Dict[str, List[Any]] = {"st": [], "cm": [], "cv": [], "cb": []}
        C = None
        for _, m in members:
            r = _role(m)
            if r is None:
                continue
            if C is None:
                C = m.num_classes
            if m.num_classes != C:
                continue
            roles[r].append(m)
        roles["st"] = roles["st"][:_MAX_CONS]
        roles["cm"] = roles["cm"][:_MAX_CONS]
        if roles["cv"]:  # one threshold set per launch: the first curve member's
            first = roles["cv"][0].thresholds
            roles["cv"] = [roles["cv"][0]]
            del first
        roles["cb"] = roles["cb"][:1]
        self.C = C
        self.roles = roles
        self.metrics = [m for r in ("st", "cm", "cv", "cb") for m in roles[r]]
        self.metric_ids = frozenset(id(m) for m in self.metrics)
        self.versions = tuple(m.__dict__.get("_cfg_version", 0) for m in self.metrics)
        self.ok = C is not None and len(self.metrics) >= 2  # one member alone keeps its own (native) update
        T = roles["cv"][0].thresholds.numel() if roles["cv"] else 0
        nb = roles["cb"][0].n_bins + 1 if roles["cb"] else 0
        need_cm = bool(roles["st"] or roles["cm"])
        if self.ok:
            words = (C * C if need_cm else 0) + (2 * (T + 1) * C * 2 if T else 0) + 2 * nb * 3
            self.ok = words + 2 * T + nb <= _LDS_WORDS
        self.T, self.nb, self.need_cm = T, nb, need_cm
        self.work: Optional[Tensor] = None
        self.cand: Optional[Tensor] = None
        self.slot = 0
        self.calls = 0
        # (member __dict__, attribute) of every object the cached argument lists depend on
        keys = [(m.__dict__, "confmat") for m in roles["cm"]]
        keys += [(m.__dict__, a) for m in roles["st"] for a in ("tp", "fp", "tn", "fn")]
        keys += [(m.__dict__, "confmat") for m in roles["cv"]]
        keys += [(m.__dict__, "_device_errors") for m in self.metrics]
        if roles["cv"]:  # the threshold buffer the cached (thresholds, permutation) pair was built from
            keys.append((roles["cv"][0].__dict__["_buffers"], "thresholds"))
        self._state_keys = keys
        # the same pairs as two parallel lists: map(dict.get, dicts, names) walks them at C speed
        self._sk_dicts = [d for d, _ in keys]
        self._sk_names = [a for _, a in keys]
        self._state_cache: Optional[tuple] = None

    def valid(self, members: List[Tuple[str, Any]]) -> bool:
        return all(m.__dict__.get("_cfg_version", 0) == v for m, v in zip(self.metrics, self.versions))

    def _states(self, dev: torch.device) -> Optional[tuple]:
        """The consumers' state tensors, or None when any is not an in-place target on ``dev``."""
        def ok(t: Any, n: int) -> bool:
            return (isinstance(t, Tensor) and t.device == dev and t.dtype == torch.long and t.is_contiguous()
                    and t.numel() == n)

        C = self.C
        cm, st, micro = [], [], []
        for m in self.roles["cm"]:
            if not ok(m.confmat, C * C):
                return None
            cm.append(m.confmat)
        for m in self.roles["st"]:
            n = 1 if m._micro else C
            s4 = (m.tp, m.fp, m.tn, m.fn)
            if not all(ok(s, n) for s in s4):
                return None
            st.extend(s4)
            micro.append(1 if m._micro else 0)
        curve = None
        if self.roles["cv"]:
            m = self.roles["cv"][0]
            if not ok(m.confmat, self.T * C * 4):
                return None
            curve = m.confmat
        return cm, st, micro, curve

    def run(self, preds: Any, target: Any) -> bool:
        """Update every member from ``(preds, target)`` in two launches; False (nothing done) when the inputs or
        states are off the fused path."""
        if not (isinstance(preds, Tensor) and isinstance(target, Tensor) and preds.is_cuda and target.is_cuda):
            return False
        C = self.C
        if (preds.ndim != 2 or target.ndim != 1 or preds.shape[1] != C or preds.shape[0] != target.shape[0]
                or preds.shape[0] == 0 or preds.dtype not in (torch.bfloat16, torch.float16, torch.float32)
                or target.dtype not in (torch.int64, torch.int32) or preds.device != target.device
                or (preds.requires_grad and torch.is_grad_enabled())):
            return False
        dev = preds.device
        # the consumers' state objects as of the last run: unchanged (updated in place, the common case) -> the
        # checked argument lists are reused (a per-call walk of ~40 state checks was ~8 us of host time)
        cur = list(map(dict.get, self._sk_dicts, self._sk_names))
        hit = self._state_cache
        if hit is not None and hit[0] == dev and all(map(operator.is_, hit[1], cur)):
            cm, st, micro, curve, err, thr, perm, bounds = hit[2]
        else:
            states = self._states(dev)
            if states is None:
                return False
            cm, st, micro, curve = states
            err = [m._device_error_buffer(dev) for m in self.metrics if m.validate_args]
            thr = perm = bounds = _empty(dev)
            if curve is not None:
                m = self.roles["cv"][0]
                thr, perm, _, _ = m._cws.get(m.thresholds.to(dev), C)
            if self.roles["cb"]:
                bounds = self.roles["cb"][0]._bounds(dev)
            # (re-read: _device_error_buffer may have just created a word)
            cur = list(map(dict.get, self._sk_dicts, self._sk_names))
            self._state_cache = (dev, cur, (cm, st, micro, curve, err, thr, perm, bounds))
        preds, target = preds.contiguous(), target.contiguous()
        n = preds.shape[0]
        if self.work is None or self.work.device != dev:
            words = int(ops._ops().mc_family_work_words(C, self.need_cm, self.T, self.nb))
            self.work = torch.zeros(words, dtype=torch.int32, device=dev)  # zero once: every fold re-zeroes it
            self.slot = 0
        empty = _empty(dev)
        conf = acc = bins = empty
        cb = self.roles["cb"][0] if self.roles["cb"] else None
        cache = None
        if cb is not None:
            conf = torch.empty(n, dtype=torch.float32, device=dev)
            acc = torch.empty(n, dtype=torch.float32, device=dev)
            if self.cand is None or self.cand.device != dev or self.cand.numel() < 4 * n:
                self.cand = torch.empty(4 * max(n, 1024), dtype=torch.float32, device=dev)
            cache = _calibration_cache(cb, dev)
            if cache is not None:
                bins = cache[0]
        ops._fast().mc_family_update(preds, target, cm, st, micro, curve if curve is not None else empty, thr, perm,
                                     conf, acc, bounds, bins, err, self.work, self.slot,
                                     self.cand if cb is not None else empty)
        if not torch.cuda.is_current_stream_capturing():  # captured: the kernel side runs the one-word protocol
            self.slot ^= 1
        self.calls += 1
        for m in self.metrics:
            d = m.__dict__
            d["_computed"] = None
            d["_update_count"] += 1
        if cb is not None:
            cb.confidences.append(conf)
            cb.accuracies.append(acc)
            if cache is not None:
                cache[1] += n
        return True


_EMPTY: Dict[Any, Tensor] = {}


def _empty(dev: torch.device) -> Tensor:
    key = (dev.type, dev.index)
    t = _EMPTY.get(key)
    if t is None:
        t = _EMPTY[key] = torch.empty(0, dtype=torch.int32, device=dev)
    return t


def _calibration_cache(m: Any, dev: torch.device) -> Optional[list]:
    """What ``_BinnedCalibration._cache_add`` would do before this batch's bins are added: the cache entry to add into
    (created for a metric with no samples yet), or None (and any stale cache dropped)."""
    if m.n_bins + 1 > 4096:
        m.__dict__.pop("_bin_cache", None)
        return None
    cache = m.__dict__.get("_bin_cache")
    if cache is None or cache[0].device != dev or cache[2] is not m.confidences:
        if m._list_numel() != 0:
            m.__dict__.pop("_bin_cache", None)
            return None
        cache = [torch.zeros(m.n_bins + 1, 3, dtype=torch.float32, device=dev), 0, m.confidences]
        m.__dict__["_bin_cache"] = cache
    return cache


__all__ = ["FamilyPlan"]
