"""Correlation / similarity / divergence regression metrics, functional API.

Parity: reference ``F/regression/{pearson,concordance,spearman,kendall,cosine_similarity,kl_divergence}.py``.

* Pearson / concordance: the update folds a batch into running (mean, M2, co-moment) states from one pass of the
  fused moments kernel with the running means as shifts -- no ``num_prior.mean() > 0`` host branch (reference
  ``F/regression/pearson.py:56``) and no separate mean/var passes.
* Spearman: vectorised average-rank with ties (sort + segment means) instead of the reference's Python loop over
  repeated values (``F/regression/spearman.py:42-50``).
* Kendall: concordant / discordant counts in O(n log^2 n) (lexicographic sort + merge-sort inversion count,
  batched over columns) instead of the reference's O(n^2) Python loop over i (``F/regression/kendall.py:61-85``).
"""
import math
from typing import Optional, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.functional.regression.streaming import _check_data_shape_to_num_outputs
from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.compute import _safe_xlogy
from torchmetrics_amd.utilities.enums import EnumStr
from torchmetrics_amd.utilities.prints import rank_zero_warn
from torchmetrics_amd.utils.deferred import warn_if


# ----------------------------------------------------------------------------------------------------------- Pearson
def _pearson_corrcoef_update(
    preds: Tensor,
    target: Tensor,
    mean_x: Tensor,
    mean_y: Tensor,
    var_x: Tensor,
    var_y: Tensor,
    corr_xy: Tensor,
    num_prior: Tensor,
    num_outputs: int,
    sink: Optional[list] = None,
) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """Fold one batch into the running (mean, sum of squared deviations, co-moment, count) states."""
    _check_same_shape(preds, target)
    _check_data_shape_to_num_outputs(preds, target, num_outputs)
    k = num_outputs
    n = preds.shape[0]
    shift_x = mean_x.reshape(k).float().contiguous()
    shift_y = mean_y.reshape(k).float().contiguous()
    states = (mean_x, mean_y, var_x, var_y, corr_xy, num_prior)
    if preds.is_cuda and all(
        t.is_cuda and t.dtype in (torch.float32, torch.float64) and t.numel() == k and t.is_contiguous() for t in states
    ) and not (torch.is_grad_enabled() and (preds.requires_grad or target.requires_grad)) and len(
        {t.data_ptr() for t in states}
    ) == 6:
        # the whole fold runs on the device inside the update's launch(es), states updated in place; a
        # ``MetricCollection`` may defer it (``sink``) to merge it with its other streaming regression members
        plan = ops.MomentsPlan(preds.reshape(n, k), target.reshape(n, k), k, [], [], fold_states=list(states),
                               shift_p=shift_x, shift_t=shift_y)
        if sink is not None and plan.deferrable():
            sink.append(plan)
        else:
            plan.run()
        return states
    s = ops.moments_update(preds.reshape(n, k), target.reshape(n, k), k, [ops.SP, ops.ST, ops.SPP, ops.STT, ops.SPT],
                           [], [], shift_p=shift_x, shift_t=shift_y, want_sums=True)
    sd, se = s[:, ops.SP], s[:, ops.ST]
    sdd, see, sde = s[:, ops.SPP], s[:, ops.STT], s[:, ops.SPT]
    n0 = num_prior.double()
    tot = n0 + n
    dx = sd / tot  # mean_x_new - mean_x
    dy = se / tot
    dt = mean_x.dtype
    new_mean_x = mean_x + dx.to(dt)
    new_mean_y = mean_y + dy.to(dt)
    new_var_x = var_x + (sdd - dx * sd).to(dt)
    new_var_y = var_y + (see - dy * se).to(dt)
    new_corr = corr_xy + (sde - dx * se).to(dt)
    return new_mean_x, new_mean_y, new_var_x, new_var_y, new_corr, num_prior + n


_LOW_VAR_WARNING = (
    "The variance of predictions or target is close to zero. This can cause instability in Pearson correlation"
    "coefficient, leading to wrong results. Consider re-scaling the input if possible or computing using a"
    "larger dtype (currently using {}).")


def _fused_corr(kind: int, mean_x: Optional[Tensor], mean_y: Optional[Tensor], var_x: Tensor, var_y: Tensor,
                corr_xy: Tensor, nb: Tensor) -> Optional[Tensor]:
    """Pearson / concordance of ROCm f32 / f64 states in one launch (None: not eligible)."""
    if not var_x.is_cuda:
        return None
    states = (mean_x if mean_x is not None else var_x, mean_y if mean_y is not None else var_y, var_x, var_y, corr_xy)
    if not ops.regression_computable(states, nb):
        return None
    bound = math.sqrt(torch.finfo(var_x.dtype).eps)
    out = ops.regression_compute(kind, states, nb, 0, bound)
    k = var_x.numel()
    warn_if(out[k + 1], _LOW_VAR_WARNING.format(var_x.dtype))
    return out[:k].view(var_x.shape)


def _pearson_corrcoef_compute(var_x: Tensor, var_y: Tensor, corr_xy: Tensor, nb: Tensor) -> Tensor:
    fused = _fused_corr(ops.REG_PEARSON, None, None, var_x, var_y, corr_xy, nb)
    if fused is not None:
        return fused.squeeze()
    var_x = var_x / (nb - 1)
    var_y = var_y / (nb - 1)
    corr_xy = corr_xy / (nb - 1)
    if var_x.dtype == torch.float16 and var_x.device == torch.device("cpu"):
        var_x, var_y = var_x.bfloat16(), var_y.bfloat16()
    bound = math.sqrt(torch.finfo(var_x.dtype).eps)
    if (var_x < bound).any() or (var_y < bound).any():
        rank_zero_warn(_LOW_VAR_WARNING.format(var_x.dtype), UserWarning)
    corr = (corr_xy / (var_x * var_y).sqrt()).squeeze()
    return torch.clamp(corr, -1.0, 1.0)


def _final_aggregation(
    means_x: Tensor, means_y: Tensor, vars_x: Tensor, vars_y: Tensor, corrs_xy: Tensor, nbs: Tensor
) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """Merge per-rank ``[W, k]`` running statistics (Chan et al. parallel update, equivalent to the reference's
    ``S/regression/pearson.py:28-71`` loop over ranks): ONE ``ops.corr_merge`` launch over the stacked states (fp64
    arithmetic, one rounding to the states' dtype), a host fold of the same formula when the library is absent."""
    states = (means_x, means_y, vars_x, vars_y, corrs_xy, nbs)
    dt = means_x.dtype
    if (dt in (torch.float32, torch.float64) and ops.native_available()
            and all(t.dtype == dt and t.shape == means_x.shape and t.device == means_x.device for t in states)):
        w = means_x.shape[0]
        merged = ops.corr_merge(torch.stack(states).reshape(6, w, -1))
        tail = means_x.shape[1:]
        return tuple(merged[i].view(tail) for i in range(6))  # type: ignore[return-value]
    mx, my, vx, vy, cxy, n = means_x[0], means_y[0], vars_x[0], vars_y[0], corrs_xy[0], nbs[0]
    for i in range(1, len(means_x)):
        mx2, my2, vx2, vy2, cxy2, n2 = means_x[i], means_y[i], vars_x[i], vars_y[i], corrs_xy[i], nbs[i]
        tot = n + n2
        dx, dy = mx2 - mx, my2 - my
        w = n * n2 / tot
        vx = vx + vx2 + dx * dx * w
        vy = vy + vy2 + dy * dy * w
        cxy = cxy + cxy2 + dx * dy * w
        mx = mx + dx * n2 / tot
        my = my + dy * n2 / tot
        n = tot
    return mx, my, vx, vy, cxy, n


def pearson_corrcoef(preds: Tensor, target: Tensor) -> Tensor:
    d = preds.shape[1] if preds.ndim == 2 else 1
    z = torch.zeros(d, dtype=preds.dtype if preds.is_floating_point() else torch.float32, device=preds.device)
    _, _, vx, vy, cxy, n = _pearson_corrcoef_update(preds, target, *(z.clone() for _ in range(6)), num_outputs=d)
    return _pearson_corrcoef_compute(vx, vy, cxy, n)


def _concordance_corrcoef_compute(
    mean_x: Tensor, mean_y: Tensor, var_x: Tensor, var_y: Tensor, corr_xy: Tensor, nb: Tensor
) -> Tensor:
    fused = _fused_corr(ops.REG_CONCORDANCE, mean_x, mean_y, var_x, var_y, corr_xy, nb)
    if fused is not None:
        return fused
    pearson = _pearson_corrcoef_compute(var_x, var_y, corr_xy, nb)
    vx, vy = var_x / (nb - 1), var_y / (nb - 1)
    return 2.0 * pearson * vx.sqrt() * vy.sqrt() / (vx + vy + (mean_x - mean_y) ** 2)


def concordance_corrcoef(preds: Tensor, target: Tensor) -> Tensor:
    d = preds.shape[1] if preds.ndim == 2 else 1
    z = torch.zeros(d, dtype=preds.dtype if preds.is_floating_point() else torch.float32, device=preds.device)
    mx, my, vx, vy, cxy, n = _pearson_corrcoef_update(preds, target, *(z.clone() for _ in range(6)), num_outputs=d)
    return _concordance_corrcoef_compute(mx, my, vx, vy, cxy, n)  # [1] for 1-D inputs, as the reference


# ---------------------------------------------------------------------------------------------------------- Spearman
def _rank_data(data: Tensor) -> Tensor:
    """1-based ranks along dim 0 with ties given their average rank (vectorised).

    On ROCm: one sorted-run launch chain for all columns (``csrc/sort/clf_curve.hip`` average-rank emission: radix
    sort with the flat id as payload, tie-run scan, scatter of the run's mean position).
    """
    n = data.shape[0]
    if data.is_cuda and n > 0 and data.is_floating_point():
        from torchmetrics_amd.functional.classification import _sorted

        x = data if data.ndim == 2 else data.reshape(n, -1)
        k = x.shape[1]
        dummy = torch.zeros(n, dtype=torch.uint8, device=data.device)
        desc = _sorted.column_stats(x, dummy, ops.CLF_T_BINARY, emit=ops.EMIT_RANKS)[4].view(k, n).t()
        return ((n + 1) - desc).reshape(data.shape).to(data.dtype)
    sorted_vals, order = torch.sort(data, dim=0, stable=True)
    pos = torch.arange(1, n + 1, dtype=torch.float64, device=data.device)
    pos = pos.view(-1, *([1] * (data.ndim - 1))).expand_as(sorted_vals)
    new_group = torch.ones_like(sorted_vals, dtype=torch.bool)
    new_group[1:] = sorted_vals[1:] != sorted_vals[:-1]
    gid = torch.cumsum(new_group.long(), dim=0) - 1  # group index per sorted position
    cols = 1 if data.ndim == 1 else data.shape[1]
    g2 = gid.reshape(n, cols)
    offs = torch.arange(cols, device=data.device) * n
    flat_gid = (g2 + offs).reshape(-1)
    sums = torch.zeros(n * cols, dtype=torch.float64, device=data.device).index_add_(0, flat_gid, pos.reshape(n, cols).reshape(-1))
    cnts = torch.zeros(n * cols, dtype=torch.float64, device=data.device).index_add_(
        0, flat_gid, torch.ones(n * cols, dtype=torch.float64, device=data.device))
    avg = (sums / cnts.clamp(min=1))[flat_gid].reshape(n, cols)
    ranks = torch.empty(n, cols, dtype=torch.float64, device=data.device)
    ranks.scatter_(0, order.reshape(n, cols), avg)
    return ranks.reshape(data.shape).to(data.dtype)


def _spearman_corrcoef_update(preds: Tensor, target: Tensor, num_outputs: int) -> Tuple[Tensor, Tensor]:
    if not (preds.is_floating_point() and target.is_floating_point()):
        raise TypeError(
            "Expected `preds` and `target` both to be floating point tensors,"
            f" but got {preds.dtype} and {target.dtype}"
        )
    _check_same_shape(preds, target)
    _check_data_shape_to_num_outputs(preds, target, num_outputs)
    return preds, target


def _spearman_corrcoef_compute(preds: Tensor, target: Tensor, eps: float = 1e-6) -> Tensor:
    preds = _rank_data(preds)
    target = _rank_data(target)
    pd = preds - preds.mean(0)
    td = target - target.mean(0)
    cov = (pd * td).mean(0)
    ps = torch.sqrt((pd * pd).mean(0))
    ts = torch.sqrt((td * td).mean(0))
    return torch.clamp(cov / (ps * ts + eps), -1.0, 1.0)


def spearman_corrcoef(preds: Tensor, target: Tensor) -> Tensor:
    preds, target = _spearman_corrcoef_update(preds, target, num_outputs=1 if preds.ndim == 1 else preds.shape[-1])
    return _spearman_corrcoef_compute(preds, target)


# ----------------------------------------------------------------------------------------------------------- Kendall
class _MetricVariant(EnumStr):
    A = "a"
    B = "b"
    C = "c"

    @staticmethod
    def _name() -> str:
        return "variant"


class _TestAlternative(EnumStr):
    TWO_SIDED = "two-sided"
    LESS = "less"
    GREATER = "greater"

    @staticmethod
    def _name() -> str:
        return "alternative"


def _tied_pairs(sorted_vals: Tensor, *more: Tensor) -> Tensor:
    """Per column of ``[n, k]`` columns sorted so equal keys are adjacent: the number of pairs with equal keys
    (sum over runs of t (t - 1) / 2), from each element's position inside its run."""
    n = sorted_vals.shape[0]
    if n < 2:
        return torch.zeros(sorted_vals.shape[1], dtype=torch.int64, device=sorted_vals.device)
    eq = sorted_vals[1:] == sorted_vals[:-1]
    for m in more:
        eq &= m[1:] == m[:-1]
    idx = torch.arange(n, device=sorted_vals.device).unsqueeze(1).expand(n, sorted_vals.shape[1])
    new_run = torch.ones_like(idx, dtype=torch.bool)
    new_run[1:] = ~eq
    start = torch.cummax(torch.where(new_run, idx, torch.zeros_like(idx)), dim=0).values
    return (idx - start).sum(0)


def _pair_counts(x: Tensor, y: Tensor) -> Tuple[Tensor, Tensor]:
    """Concordant / discordant pair counts per column of ``[n, k]`` inputs in O(n log^2 n) (Knight's method).

    Sort lexicographically by (x, y); the discordant pairs are then exactly the strict inversions of the y sequence
    (pairs tied in x are ordered by y, pairs tied in y are not inversions), counted by a bottom-up merge sort whose
    every pass is one batched ``searchsorted`` (right-run elements vs the sorted left run) + one batched sort.  The
    concordant count follows from n(n-1)/2 - ties(x) - ties(y) + joint ties - discordant.  The reference compares all
    pairs with a Python loop over i (``F/regression/kendall.py:61-85``)."""
    n, k = x.shape
    if n < 2:
        z = torch.zeros(k, dtype=torch.int64, device=x.device)
        return z, z.clone()
    o1 = torch.argsort(y, dim=0, stable=True)
    ys1 = torch.gather(y, 0, o1)
    o2 = torch.argsort(torch.gather(x, 0, o1), dim=0, stable=True)
    order = torch.gather(o1, 0, o2)
    xs, ys = torch.gather(x, 0, order), torch.gather(y, 0, order)
    size = 1 << (n - 1).bit_length()
    seq = ys.t().double()
    if size > n:
        seq = torch.cat([seq, seq.new_full((k, size - n), float("inf"))], 1)
    disc = torch.zeros(k, dtype=torch.int64, device=x.device)
    w = 1
    while w < size:
        blocks = seq.reshape(k, size // (2 * w), 2, w)
        left, right = blocks[:, :, 0].contiguous(), blocks[:, :, 1].contiguous()
        disc += (w - torch.searchsorted(left, right, right=True)).sum(dim=(1, 2))
        seq = torch.sort(blocks.reshape(k, size // (2 * w), 2 * w), dim=-1).values.reshape(k, size)
        w *= 2
    pairs = n * (n - 1) // 2
    conc = pairs - _tied_pairs(xs) - _tied_pairs(ys1) + _tied_pairs(xs, ys) - disc
    return conc, disc


def _pair_counts_allpairs(x: Tensor, y: Tensor, chunk: int = 2048) -> Tuple[Tensor, Tensor]:
    """O(n^2) chunked all-pairs reference of :func:`_pair_counts` (kept for tests)."""
    n = x.shape[0]
    conc = torch.zeros(x.shape[1], dtype=torch.int64, device=x.device)
    disc = torch.zeros_like(conc)
    idx = torch.arange(n, device=x.device)
    for s in range(0, n, chunk):
        xi, yi = x[s : s + chunk].unsqueeze(1), y[s : s + chunk].unsqueeze(1)  # [c,1,k]
        upper = (idx[s : s + chunk].unsqueeze(1) < idx.unsqueeze(0)).unsqueeze(-1)  # j > i
        dx = torch.sign(x.unsqueeze(0) - xi)
        dy = torch.sign(y.unsqueeze(0) - yi)
        prod = dx * dy
        conc += ((prod > 0) & upper).sum((0, 1))
        disc += ((prod < 0) & upper).sum((0, 1))
    return conc, disc


def _tie_stats(x: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """Per column: Σ t(t-1)/2, Σ t(t-1)(t-2), Σ t(t-1)(2t+5) over tie groups of size t."""
    out = []
    for c in range(x.shape[1]):
        _, cnt = torch.unique(x[:, c], return_counts=True)
        cnt = cnt[cnt > 1].double()
        out.append(torch.stack([(cnt * (cnt - 1) / 2).sum(), (cnt * (cnt - 1) * (cnt - 2)).sum(),
                                (cnt * (cnt - 1) * (2 * cnt + 5)).sum()]))
    st = torch.stack(out, 1).to(x.device)
    return st[0], st[1], st[2]


def _kendall_corrcoef_update(preds: Tensor, target: Tensor, concat_preds=None, concat_target=None,  # noqa: ANN001
                             num_outputs: int = 1) -> Tuple[list, list]:
    _check_same_shape(preds, target)
    _check_data_shape_to_num_outputs(preds, target, num_outputs)
    if num_outputs == 1:
        preds, target = preds.unsqueeze(1), target.unsqueeze(1)
    concat_preds = (concat_preds or []) + [preds]
    concat_target = (concat_target or []) + [target]
    return concat_preds, concat_target


def _kendall_corrcoef_compute(
    preds: Tensor, target: Tensor, variant: _MetricVariant, alternative: Optional[_TestAlternative] = None
) -> Tuple[Tensor, Optional[Tensor]]:
    if preds.ndim == 1:
        preds, target = preds.unsqueeze(1), target.unsqueeze(1)
    n = preds.shape[0]
    # one stats launch chain (ROCm: csrc/sort/kendall.hip) -> discordant pairs, tie terms, distinct counts
    st = ops.kendall_stats(preds, target)
    disc, pt, pt1, pt2, tt, tt1, tt2, txy, pu, tu = st.to(preds.device).unbind(1)
    nt = torch.tensor(float(n), dtype=torch.float64, device=preds.device)
    conc = nt * (nt - 1) / 2 - pt - tt + txy - disc
    cmd = conc - disc
    if variant == _MetricVariant.A:
        tau = cmd / (conc + disc)
    elif variant == _MetricVariant.B:
        tot = nt * (nt - 1) / 2
        tau = cmd / torch.sqrt((tot - pt) * (tot - tt))
    else:
        m = torch.minimum(pu, tu)
        tau = 2 * cmd / ((m - 1) / m * nt**2)
    p_value = None
    if alternative is not None:
        base = nt * (nt - 1) * (2 * nt + 5)
        if variant == _MetricVariant.A:
            t_val = 3 * cmd / torch.sqrt(base / 2)
        else:
            m2 = nt * (nt - 1)
            den = (base - pt2 - tt2) / 18 + (2 * pt * tt) / m2 + pt1 * tt1 / (9 * m2 * (nt - 2))
            t_val = cmd / torch.sqrt(den)
        if alternative == _TestAlternative.TWO_SIDED:
            t_val = torch.abs(t_val)
        if alternative in (_TestAlternative.TWO_SIDED, _TestAlternative.GREATER):
            t_val = -t_val
        nan = torch.isnan(t_val)
        p_value = torch.distributions.Normal(0.0, 1.0).cdf(torch.nan_to_num(t_val).float().cpu()).to(preds.device)
        p_value = torch.where(nan, torch.full_like(p_value, float("nan")), p_value)
        if alternative == _TestAlternative.TWO_SIDED:
            p_value = p_value * 2
        p_value = p_value.clamp(max=1.0) if alternative == _TestAlternative.TWO_SIDED else p_value
        p_value = p_value.squeeze().to(preds.dtype if preds.is_floating_point() else torch.float32)
    tau = tau.squeeze().to(preds.dtype if preds.is_floating_point() else torch.float32)
    return tau, p_value


def kendall_rank_corrcoef(
    preds: Tensor,
    target: Tensor,
    variant: str = "b",
    t_test: bool = False,
    alternative: Optional[str] = "two-sided",
) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    if not isinstance(t_test, bool):
        raise ValueError(f"Argument `t_test` is expected to be of a type `bool`, but got {type(t_test)}.")
    if t_test and alternative is None:
        raise ValueError("Argument `alternative` is required if `t_test=True` but got `None`.")
    _variant = _MetricVariant.from_str(str(variant))
    _alternative = _TestAlternative.from_str(str(alternative)) if t_test else None
    _check_same_shape(preds, target)
    tau, p = _kendall_corrcoef_compute(preds, target, _variant, _alternative)
    return (tau, p) if p is not None else tau


# ------------------------------------------------------------------------------------------------- cosine similarity
def _cosine_similarity_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    _check_same_shape(preds, target)
    if preds.ndim != 2:
        raise ValueError(
            "Expected input to cosine similarity to be 2D tensors of shape `[N,D]` where `N` is the number of samples"
            f" and `D` is the number of dimensions, but got tensor of shape {preds.shape}"
        )
    # at least fp32 (the reference casts to fp32 unconditionally; fp64 inputs keep their precision here)
    dt = torch.promote_types(torch.promote_types(preds.dtype, target.dtype), torch.float32)
    return preds.to(dt), target.to(dt)


def _cosine_similarity_compute(preds: Tensor, target: Tensor, reduction: Optional[str] = "sum") -> Tensor:
    dot = (preds * target).sum(dim=-1)
    sim = dot / (preds.norm(dim=-1) * target.norm(dim=-1))
    red = {"sum": torch.sum, "mean": torch.mean, "none": lambda x: x, None: lambda x: x}
    return red[reduction](sim)


def cosine_similarity(preds: Tensor, target: Tensor, reduction: Optional[str] = "sum") -> Tensor:
    return _cosine_similarity_compute(*_cosine_similarity_update(preds, target), reduction)


# ------------------------------------------------------------------------------------------------------ KL divergence
def _kld_update(p: Tensor, q: Tensor, log_prob: bool) -> Tuple[Tensor, int]:
    _check_same_shape(p, q)
    if p.ndim != 2 or q.ndim != 2:
        raise ValueError(f"Expected both p and q distribution to be 2D but got {p.ndim} and {q.ndim} respectively")
    total = p.shape[0]
    if log_prob:
        measures = torch.sum(p.exp() * (p - q), dim=-1)
    else:
        p = p / p.sum(dim=-1, keepdim=True)
        q = q / q.sum(dim=-1, keepdim=True)
        measures = _safe_xlogy(p, p / q).sum(dim=-1)
    return measures, total


def _kld_compute(measures: Tensor, total: Union[int, Tensor], reduction: Optional[str] = "mean") -> Tensor:
    if reduction == "sum":
        return measures.sum()
    if reduction == "mean":
        return measures.sum() / total
    if reduction is None or reduction == "none":
        return measures
    return measures / total


def kl_divergence(p: Tensor, q: Tensor, log_prob: bool = False, reduction: Optional[str] = "mean") -> Tensor:
    measures, total = _kld_update(p, q, log_prob)
    return _kld_compute(measures, total, reduction)
