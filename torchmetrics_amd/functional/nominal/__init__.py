"""Nominal (categorical) association metrics (reference ``F/nominal/{cramers,tschuprows,pearson,theils_u,
fleiss_kappa,utils}.py``).

MI355X-first design: every statistic is evaluated on a *batch* of contingency tables ``[B, K, K]`` with empty rows /
columns masked instead of physically dropped, so the ``*_matrix`` variants build all ``V (V - 1) / 2`` pairwise tables
with ONE histogram launch (keys ``pair * K^2 + y * K + x`` into the HIP LDS histogram, :func:`ops.histogram`) and
evaluate them in one vectorised pass -- the reference loops over ``itertools.combinations`` and pays a
``unique`` + bincount + host sync per pair (``F/nominal/cramers.py:175-182``).
"""
import itertools
from typing import Literal, Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.utilities.prints import rank_zero_warn

_NanStrategy = Literal["replace", "drop"]
# pairs per histogram launch is bounded so the key tensor stays below this many elements
_MAX_KEYS = 1 << 27


# --------------------------------------------------------------------------------------------------- helpers
def _nominal_input_validation(nan_strategy: str, nan_replace_value: Optional[float]) -> None:
    if nan_strategy not in ["replace", "drop"]:
        raise ValueError(
            f"Argument `nan_strategy` is expected to be one of `['replace', 'drop']`, but got {nan_strategy}"
        )
    if nan_strategy == "replace" and not isinstance(nan_replace_value, (float, int)):
        raise ValueError(
            "Argument `nan_replace` is expected to be of a type `int` or `float` when `nan_strategy = 'replace`, "
            f"but got {nan_replace_value}"
        )


def _handle_nan_in_data(preds: Tensor, target: Tensor, nan_strategy: _NanStrategy = "replace",
                        nan_replace_value: Optional[float] = 0.0) -> Tuple[Tensor, Tensor]:
    if nan_strategy == "replace":
        return preds.nan_to_num(nan_replace_value), target.nan_to_num(nan_replace_value)
    keep = ~torch.logical_or(preds.isnan(), target.isnan())
    return preds[keep], target[keep]


def _drop_empty_rows_and_cols(confmat: Tensor) -> Tensor:
    confmat = confmat[confmat.sum(1) != 0]
    return confmat[:, confmat.sum(0) != 0]


def _nominal_confmat(preds: Tensor, target: Tensor, num_classes: int, nan_strategy: _NanStrategy = "replace",
                     nan_replace_value: Optional[float] = 0.0, flag: Optional[Tensor] = None) -> Tensor:
    """``[num_classes, num_classes]`` table ``cm[target, preds]`` (one-hot / prob inputs are arg-maxed)."""
    preds = preds.argmax(1) if preds.ndim == 2 else preds
    target = target.argmax(1) if target.ndim == 2 else target
    preds, target = _handle_nan_in_data(preds, target, nan_strategy, nan_replace_value)
    p, t = preds.long(), target.long()
    if flag is not None:
        bad = (p < 0) | (p >= num_classes) | (t < 0) | (t >= num_classes)
        flag.bitwise_or_(bad.any().to(torch.int32) * 1)  # TARGET_OUT_OF_RANGE, raised at compute
    elif p.numel() and not p.is_cuda and (min(p.min(), t.min()) < 0 or max(p.max(), t.max()) >= num_classes):
        raise ValueError(f"Expected nominal values in [0, {num_classes}), found values outside that range.")
    keys = torch.where((p >= 0) & (p < num_classes) & (t >= 0) & (t < num_classes), t * num_classes + p, -1)
    return ops.histogram(keys, num_classes * num_classes).reshape(num_classes, num_classes)


def _num_classes_of(preds: Tensor, target: Tensor) -> int:
    """Class count covering every observed value (empty rows/cols are masked, so over-sizing is harmless)."""
    both = torch.cat([preds.flatten(), target.flatten()])
    both = both[~both.isnan()] if both.is_floating_point() else both
    return int(both.max().item()) + 1 if both.numel() else 1


class _TableStats:
    """Statistics of a batch of contingency tables ``cm[B, R, C]`` with empty rows / columns masked (equal to those
    of the compacted tables the reference builds, ``F/nominal/utils.py:34-59``).  ROCm: one block per table
    (``ops.nominal_table_stats``, fp64); else the same quantities with masked torch ops."""

    def __init__(self, cm: Tensor) -> None:
        st = ops.nominal_table_stats(cm) if cm.shape[-1] == cm.shape[-2] else None
        if st is None:
            st = self._torch_stats(cm.to(torch.float64))
        self.n, self.r, self.c = st[:, 0], st[:, 1], st[:, 2]
        self._chi, self._chi_yates, self.s_xy, self.s_x = st[:, 3], st[:, 4], st[:, 5], st[:, 6]

    @staticmethod
    def _torch_stats(cm: Tensor) -> Tensor:
        rs, cs = cm.sum(2), cm.sum(1)
        rowm, colm = rs > 0, cs > 0
        n = cm.sum((1, 2))
        valid = rowm[:, :, None] & colm[:, None, :]
        exp = rs[:, :, None] * cs[:, None, :] / n[:, None, None].clamp(min=1)
        safe_exp = torch.where(valid, exp, torch.ones_like(exp))
        zero = torch.zeros_like(exp)
        chi = torch.where(valid, (cm - exp) ** 2 / safe_exp, zero).sum((1, 2))
        yates = cm + 0.5 * torch.sign(exp - cm)
        chi_y = torch.where(valid, (yates - exp) ** 2 / safe_exp, zero).sum((1, 2))
        nz = cm > 0
        ratio = rs[:, :, None] / torch.where(nz, cm, torch.ones_like(cm))
        s_xy = torch.where(nz, cm / n[:, None, None].clamp(min=1) * torch.log(ratio), zero).sum((1, 2))
        p_x = cs / n[:, None].clamp(min=1)
        s_x = -torch.where(colm, p_x * torch.log(torch.where(colm, p_x, torch.ones_like(p_x))),
                           torch.zeros_like(p_x)).sum(1)
        r, c = rowm.sum(1).to(torch.float64), colm.sum(1).to(torch.float64)
        return torch.stack([n, r, c, chi, chi_y, s_xy, s_x, torch.zeros_like(n)], 1)

    def chi_squared(self, bias_correction: bool) -> Tensor:
        """Pearson chi^2 with Yates continuity correction for 2x2 tables (scipy ``chi2_contingency`` semantics)."""
        df = (self.r - 1) * (self.c - 1)
        chi = torch.where(df == 1, self._chi_yates, self._chi) if bias_correction else self._chi
        return torch.where(df == 0, torch.zeros_like(df), chi)

    def bias_corrected(self, phi2: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
        n1 = self.n - 1
        phi2c = torch.clamp(phi2 - (self.r - 1) * (self.c - 1) / n1, min=0.0)
        return phi2c, self.r - (self.r - 1) ** 2 / n1, self.c - (self.c - 1) ** 2 / n1


def _bias_nan(value: Tensor, rc: Tensor, cc: Tensor, name: str) -> Tensor:
    degenerate = torch.minimum(rc, cc) == 1
    if bool(degenerate.any()):
        rank_zero_warn(f"Unable to compute {name} using bias correction. Please consider to set `bias_correction=False`.")
    return torch.where(degenerate, torch.full_like(value, float("nan")), value)


def _cramers_v_batched(cm: Tensor, bias_correction: bool) -> Tensor:
    st = _TableStats(cm)
    phi2 = st.chi_squared(bias_correction) / st.n
    if bias_correction:
        phi2c, rc, cc = st.bias_corrected(phi2)
        v = _bias_nan(torch.sqrt(phi2c / torch.minimum(rc - 1, cc - 1)), rc, cc, "Cramer's V")
    else:
        v = torch.sqrt(phi2 / torch.minimum(st.r - 1, st.c - 1))
    return v.clamp(0.0, 1.0).to(torch.float32)


def _tschuprows_t_batched(cm: Tensor, bias_correction: bool) -> Tensor:
    st = _TableStats(cm)
    phi2 = st.chi_squared(bias_correction) / st.n
    if bias_correction:
        phi2c, rc, cc = st.bias_corrected(phi2)
        v = _bias_nan(torch.sqrt(phi2c / torch.sqrt((rc - 1) * (cc - 1))), rc, cc, "Tschuprow's T")
    else:
        v = torch.sqrt(phi2 / torch.sqrt((st.r - 1) * (st.c - 1)))
    return v.clamp(0.0, 1.0).to(torch.float32)


def _pearsons_batched(cm: Tensor) -> Tensor:
    st = _TableStats(cm)
    phi2 = st.chi_squared(False) / st.n
    return torch.sqrt(phi2 / (1 + phi2)).clamp(0.0, 1.0).to(torch.float32)


def _theils_u_batched(cm: Tensor) -> Tensor:
    """U(X|Y) with X = columns (preds), Y = rows (target): (H(X) - H(X|Y)) / H(X)."""
    st = _TableStats(cm)
    s_x, s_xy = st.s_x, st.s_xy
    u = torch.where(s_x == 0, torch.zeros_like(s_x), (s_x - s_xy) / torch.where(s_x == 0, torch.ones_like(s_x), s_x))
    return u.to(torch.float32)


def _pairwise_confmats(matrix: Tensor, nan_strategy: _NanStrategy, nan_replace_value: Optional[float],
                       pairs: Tensor) -> Tuple[Tensor, int]:
    """All pairwise tables ``cm[p] [y = col j, x = col i]`` for ``pairs [P, 2]`` with chunked histogram launches."""
    m = matrix.nan_to_num(nan_replace_value) if nan_strategy == "replace" else matrix
    finite = ~m.isnan() if m.is_floating_point() else torch.ones_like(m, dtype=torch.bool)
    k = int(torch.where(finite, m, torch.zeros_like(m)).max().item()) + 1 if m.numel() else 1
    mk = torch.where(finite, m, torch.zeros_like(m)).long()
    n = m.shape[0]
    out = []
    chunk = max(1, _MAX_KEYS // max(n, 1))
    for s in range(0, pairs.shape[0], chunk):
        pi, pj = pairs[s:s + chunk, 0], pairs[s:s + chunk, 1]
        x, y = mk[:, pi], mk[:, pj]  # [N, P]
        ok = finite[:, pi] & finite[:, pj]
        pid = torch.arange(pi.numel(), device=m.device)[None, :]
        keys = torch.where(ok, pid * k * k + y * k + x, torch.full_like(x, -1))
        out.append(ops.histogram(keys.flatten(), pi.numel() * k * k).reshape(pi.numel(), k, k))
    return torch.cat(out) if out else torch.zeros(0, k, k, dtype=torch.long, device=m.device), k


def _assoc_matrix(matrix: Tensor, nan_strategy: _NanStrategy, nan_replace_value: Optional[float], fn,
                  symmetric: bool = True) -> Tensor:
    _nominal_input_validation(nan_strategy, nan_replace_value)
    v = matrix.shape[1]
    out = torch.ones(v, v, device=matrix.device)
    if v < 2:
        return out
    pairs = torch.tensor(list(itertools.combinations(range(v), 2)), device=matrix.device)
    cms, _ = _pairwise_confmats(matrix, nan_strategy, nan_replace_value, pairs)
    vals = fn(cms)
    out[pairs[:, 0], pairs[:, 1]] = vals
    out[pairs[:, 1], pairs[:, 0]] = vals if symmetric else fn(cms.transpose(1, 2))
    return out


# ----------------------------------------------------------------------------------------------- functionals
def _cramers_v_update(preds: Tensor, target: Tensor, num_classes: int, nan_strategy: _NanStrategy = "replace",
                      nan_replace_value: Optional[float] = 0.0) -> Tensor:
    return _nominal_confmat(preds, target, num_classes, nan_strategy, nan_replace_value)


def _cramers_v_compute(confmat: Tensor, bias_correction: bool) -> Tensor:
    return _cramers_v_batched(confmat[None], bias_correction)[0]


def cramers_v(preds: Tensor, target: Tensor, bias_correction: bool = True, nan_strategy: _NanStrategy = "replace",
              nan_replace_value: Optional[float] = 0.0) -> Tensor:
    """Cramer's V association between two categorical series (``F/nominal/cramers.py``)."""
    _nominal_input_validation(nan_strategy, nan_replace_value)
    cm = _nominal_confmat(preds, target, _num_classes_of(preds, target), nan_strategy, nan_replace_value)
    return _cramers_v_compute(cm, bias_correction)


def cramers_v_matrix(matrix: Tensor, bias_correction: bool = True, nan_strategy: _NanStrategy = "replace",
                     nan_replace_value: Optional[float] = 0.0) -> Tensor:
    """Cramer's V between every pair of columns of ``matrix [N, V]``."""
    return _assoc_matrix(matrix, nan_strategy, nan_replace_value, lambda c: _cramers_v_batched(c, bias_correction))


_tschuprows_t_update = _cramers_v_update
_pearsons_contingency_coefficient_update = _cramers_v_update
_theils_u_update = _cramers_v_update


def _tschuprows_t_compute(confmat: Tensor, bias_correction: bool) -> Tensor:
    return _tschuprows_t_batched(confmat[None], bias_correction)[0]


def tschuprows_t(preds: Tensor, target: Tensor, bias_correction: bool = True, nan_strategy: _NanStrategy = "replace",
                 nan_replace_value: Optional[float] = 0.0) -> Tensor:
    """Tschuprow's T association (``F/nominal/tschuprows.py``)."""
    _nominal_input_validation(nan_strategy, nan_replace_value)
    cm = _nominal_confmat(preds, target, _num_classes_of(preds, target), nan_strategy, nan_replace_value)
    return _tschuprows_t_compute(cm, bias_correction)


def tschuprows_t_matrix(matrix: Tensor, bias_correction: bool = True, nan_strategy: _NanStrategy = "replace",
                        nan_replace_value: Optional[float] = 0.0) -> Tensor:
    """Tschuprow's T between every pair of columns."""
    return _assoc_matrix(matrix, nan_strategy, nan_replace_value, lambda c: _tschuprows_t_batched(c, bias_correction))


def _pearsons_contingency_coefficient_compute(confmat: Tensor) -> Tensor:
    return _pearsons_batched(confmat[None])[0]


def pearsons_contingency_coefficient(preds: Tensor, target: Tensor, nan_strategy: _NanStrategy = "replace",
                                     nan_replace_value: Optional[float] = 0.0) -> Tensor:
    """Pearson's contingency coefficient (``F/nominal/pearson.py``)."""
    _nominal_input_validation(nan_strategy, nan_replace_value)
    cm = _nominal_confmat(preds, target, _num_classes_of(preds, target), nan_strategy, nan_replace_value)
    return _pearsons_contingency_coefficient_compute(cm)


def pearsons_contingency_coefficient_matrix(matrix: Tensor, nan_strategy: _NanStrategy = "replace",
                                            nan_replace_value: Optional[float] = 0.0) -> Tensor:
    """Pearson's contingency coefficient between every pair of columns."""
    return _assoc_matrix(matrix, nan_strategy, nan_replace_value, _pearsons_batched)


def _theils_u_compute(confmat: Tensor) -> Tensor:
    return _theils_u_batched(confmat[None])[0]


def theils_u(preds: Tensor, target: Tensor, nan_strategy: _NanStrategy = "replace",
             nan_replace_value: Optional[float] = 0.0) -> Tensor:
    """Theil's U uncertainty coefficient U(preds | target) (``F/nominal/theils_u.py``)."""
    _nominal_input_validation(nan_strategy, nan_replace_value)
    cm = _nominal_confmat(preds, target, _num_classes_of(preds, target), nan_strategy, nan_replace_value)
    return _theils_u_compute(cm)


def theils_u_matrix(matrix: Tensor, nan_strategy: _NanStrategy = "replace",
                    nan_replace_value: Optional[float] = 0.0) -> Tensor:
    """Theil's U between every ordered pair of columns (asymmetric)."""
    return _assoc_matrix(matrix, nan_strategy, nan_replace_value, _theils_u_batched, symmetric=False)


def _fleiss_kappa_update(ratings: Tensor, mode: Literal["counts", "probs"] = "counts") -> Tensor:
    """``[n_samples, n_categories]`` rater counts.  ``probs`` input ``[N, C, R]`` is arg-maxed over C and one-hot
    encoded with C classes (the reference uses ``ratings.shape[1]`` *after* the argmax, i.e. R, which only coincides
    with C when R >= C, ``F/nominal/fleiss_kappa.py:30``)."""
    if mode == "probs":
        if ratings.ndim != 3 or not ratings.is_floating_point():
            raise ValueError(
                "If argument ``mode`` is 'probs', ratings must have 3 dimensions with the format"
                " [n_samples, n_categories, n_raters] and be floating point."
            )
        n, c, _ = ratings.shape
        idx = ratings.argmax(dim=1)  # [N, R]
        counts = torch.zeros(n, c, dtype=torch.long, device=ratings.device)
        return counts.scatter_add_(1, idx, torch.ones_like(idx))
    if mode == "counts" and (ratings.ndim != 2 or ratings.is_floating_point()):
        raise ValueError(
            "If argument ``mode`` is `counts`, ratings must have 2 dimensions with the format"
            " [n_samples, n_categories] and be none floating point."
        )
    return ratings


def _fleiss_kappa_compute(counts: Tensor) -> Tensor:
    total = counts.shape[0]
    counts = counts.to(torch.float64)
    raters = counts.sum(1).max()
    p_i = counts.sum(0) / (total * raters)
    p_j = ((counts**2).sum(1) - raters) / (raters * (raters - 1))
    pe = (p_i**2).sum()
    return ((p_j.mean() - pe) / (1 - pe + 1e-5)).to(torch.float32)


def fleiss_kappa(ratings: Tensor, mode: Literal["counts", "probs"] = "counts") -> Tensor:
    """Fleiss' kappa inter-rater agreement (``F/nominal/fleiss_kappa.py``)."""
    if mode not in ["counts", "probs"]:
        raise ValueError("Argument ``mode`` must be one of ['counts', 'probs'].")
    return _fleiss_kappa_compute(_fleiss_kappa_update(ratings, mode))


__all__ = [
    "cramers_v",
    "cramers_v_matrix",
    "fleiss_kappa",
    "pearsons_contingency_coefficient",
    "pearsons_contingency_coefficient_matrix",
    "theils_u",
    "theils_u_matrix",
    "tschuprows_t",
    "tschuprows_t_matrix",
]
