"""Replay of a ``MetricCollection``'s merged regression update (one kernel per compute group
per step, and the host cost that goes with it).

The collection's streaming regression leaders (MSE / MAE / R2 / explained variance / Pearson ...) already hand their
moments requests to one merged ``ops.moments_update`` per step (``ops.run_moments_plans``).  What remains per step is
host work: every member's ``update`` wrapper, its shape checks and plan object, then the merge.  Once a step has been
merged into ONE call, :class:`MomentsReplay` records that call (destinations, sum ids, mask, Pearson fold shifts) and
later steps with inputs of the same shape / dtype / device and unchanged members (configuration versions and state
objects) issue the recorded call directly and do each member's bookkeeping (``_update_count`` / ``_computed``), as its
own update would have.  Anything else -- other shapes, gradients, a member reconfigured, moved or reset into new state
objects -- takes the members' own updates, which run the reference's checks.

Only members whose ``update`` is their class's own and does shape-only checks qualify (the streaming regression
metrics of ``regression/streaming.py`` and ``PearsonCorrCoef`` with ``num_outputs=1`` and fp32 states).
"""
from typing import Any, List, Optional

import torch
from torch import Tensor

from torchmetrics_amd import ops


def _replayable(m: Any) -> bool:
    from torchmetrics_amd.regression.correlation import PearsonCorrCoef
    from torchmetrics_amd.regression.streaming import _MomentsMetric

    t = type(m)
    d = m.__dict__
    if d.get("compute_on_cpu") or d.get("dist_sync_on_step"):
        return False
    if isinstance(m, PearsonCorrCoef):
        return t.update is PearsonCorrCoef.update and d.get("num_outputs") == 1 and \
            all(getattr(m, s).dtype == torch.float32 for s in ("mean_x", "mean_y", "var_x", "var_y", "corr_xy",
                                                                "n_total"))
    if not isinstance(m, _MomentsMetric):
        return False
    # the class's own update (subclasses of the streaming base define theirs); one output
    return "update" in t.__dict__ and d.get("num_outputs", 1) == 1


class MomentsReplay:
    """One recorded merged moments call for ``members`` on 1-D inputs of ``shape`` / ``dtype``."""

    def __init__(self, members: List[Any], plan: "ops.MomentsPlan", preds: Tensor, target: Tensor) -> None:
        self.members = members
        self.member_ids = frozenset(id(x) for x in self.members)
        self.versions = tuple(m.__dict__.get("_cfg_version", 0) for m in members)
        self.states = [(m.__dict__, tuple((k, m.__dict__.get(k)) for k in m._defaults)) for m in members]
        self.shape, self.dtype, self.device = preds.shape, preds.dtype, preds.device
        fold = plan.fold_states is not None
        dests = list(plan.fold_states or []) + list(plan.dests)
        ids = list(plan.ids)
        mask = 0
        for i in ids:
            for j in ops._sum_ids(int(i)):
                mask |= 1 << int(j)
        if fold:
            mask |= (1 << ops.SP) | (1 << ops.ST) | (1 << ops.SPP) | (1 << ops.STT) | (1 << ops.SPT) | (1 << ops.COUNT)
        self.args = (plan.k, mask, float(plan.eps), float(plan.power), plan.shift_p, plan.shift_t, dests, ids,
                     False, ops.FOLD_PEARSON if fold else ops.FOLD_NONE)
        self.calls = 0

    def valid(self) -> bool:
        for m, v in zip(self.members, self.versions):
            if m.__dict__.get("_cfg_version", 0) != v:
                return False
        for d, pairs in self.states:
            for k, obj in pairs:
                if d.get(k) is not obj:
                    return False
        return True

    def run(self, preds: Any, target: Any) -> bool:
        if not (isinstance(preds, Tensor) and isinstance(target, Tensor)):
            return False
        if (preds.shape != self.shape or target.shape != self.shape or preds.dtype != self.dtype
                or target.dtype != self.dtype or preds.device != self.device or target.device != self.device):
            return False
        if torch.is_grad_enabled() and (preds.requires_grad or target.requires_grad):
            return False
        if not self.valid():
            return False
        k, mask, eps, power, sp, st, dests, ids, want, fold = self.args
        mod = ops._fast_mod or ops._fast()
        mod.moments_update(preds.reshape(-1, k), target.reshape(-1, k), k, mask, eps, power, sp, st, dests, ids,
                           want, fold)
        for m in self.members:
            d = m.__dict__
            d["_computed"] = None
            d["_update_count"] += 1
        self.calls += 1
        return True


def build(members: List[Any], merged: List["ops.MomentsPlan"], n_plans: int, preds: Any,
          target: Any) -> Optional[MomentsReplay]:
    """A replay for this step if it went through exactly one merged call covering one plan of every member."""
    if len(merged) != 1 or n_plans != len(members) or not members:
        return None
    if not (isinstance(preds, Tensor) and isinstance(target, Tensor) and preds.is_cuda and preds.ndim == 1
            and preds.shape == target.shape and preds.dtype == target.dtype and preds.is_floating_point()):
        return None
    if not all(_replayable(m) for m in members):
        return None
    plan = merged[0]
    if plan.preds.data_ptr() != preds.data_ptr() or plan.target.data_ptr() != target.data_ptr():
        return None  # the plan read converted copies: the replay would not see what the members did
    return MomentsReplay(members, plan, preds, target)


__all__ = ["MomentsReplay", "build"]
