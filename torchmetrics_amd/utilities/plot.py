"""matplotlib rendering behind ``Metric.plot`` (same call signatures as reference ``S/utilities/plot.py``).

Structure: every public function first turns its metric values into plain *series* / *panels* (host numpy arrays,
one device->host copy per value; :func:`_series_of`, :func:`_confmat_panels`, :func:`_curve_series`) and only then
draws them, so the value handling is testable without matplotlib (which is optional, as in the reference).
"""
from itertools import product
from math import ceil, floor, sqrt
from typing import Any, Dict, List, NamedTuple, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor

from torchmetrics_amd.utilities.imports import _MATPLOTLIB_AVAILABLE

_PLOT_OUT_TYPE = Tuple[Any, Any]
_AX_TYPE = Any
_MARKER = {"marker": "o", "markersize": 10}


def _error_on_missing_matplotlib() -> None:
    if not _MATPLOTLIB_AVAILABLE:
        raise ModuleNotFoundError(
            "Plot function expects `matplotlib` to be installed. Please install with `pip install matplotlib`"
        )


def _pyplot() -> Any:
    _error_on_missing_matplotlib()
    import matplotlib

    matplotlib.use("Agg", force=False)
    import matplotlib.pyplot as plt

    return plt


def _host(v: Any) -> np.ndarray:
    return v.detach().float().cpu().numpy() if isinstance(v, Tensor) else np.asarray(v, dtype=np.float32)


class _Series(NamedTuple):
    label: Optional[str]
    x: np.ndarray
    y: np.ndarray
    line: bool  # connect the points (time series) or scatter them


def _series_of(val: Any, legend_name: Optional[str] = None) -> Tuple[List[_Series], int]:
    """Metric value(s) -> drawable series, plus the number of steps when ``val`` is a history (0 otherwise).

    One value: a point.  A per-class vector: one point per class.  A dict: one point (or one series for non-scalar
    entries) per key.  A sequence of any of those: one series per class / key over the steps.
    """
    tag = (lambda i: f"{legend_name} {i}") if legend_name else str
    if isinstance(val, Tensor):
        if val.numel() == 1:
            return [_Series(None, np.zeros(1), _host(val).reshape(1), False)], 0
        return [_Series(tag(i), np.full(1, i), _host(v).reshape(-1), False) for i, v in enumerate(val)], 0
    if isinstance(val, dict):
        out, steps = [], 0
        for i, (k, v) in enumerate(val.items()):
            if v.numel() == 1:
                out.append(_Series(k, np.full(1, i), _host(v).reshape(1), False))
            else:
                y = _host(v).reshape(-1)
                out.append(_Series(k, np.arange(len(y)), y, True))
                steps = max(steps, len(y))
        return out, steps
    if isinstance(val, Sequence) and len(val) > 0:
        steps = len(val)
        xs = np.arange(steps)
        if isinstance(val[0], dict):
            return [_Series(k, xs, _host(torch.stack([step[k] for step in val])).reshape(steps), True)
                    for k in val[0]], steps
        stacked = _host(torch.stack(list(val), 0))
        if stacked.ndim == 1:
            return [_Series(None, xs, stacked, True)], steps
        return [_Series(tag(i), xs, col, True) for i, col in enumerate(stacked.reshape(steps, -1).T)], steps
    raise ValueError("Got unknown format for argument `val`.")


def _padded_limits(lo: float, hi: float, lower: Optional[float], upper: Optional[float]) -> Tuple[float, float]:
    """y-limits: the metric's bounds (or the data range) widened by 10 % of the bounded span."""
    span = (upper - lower) if (lower is not None and upper is not None) else (hi - lo)
    pad = 0.1 * span
    return (lower if lower is not None else lo) - pad, (upper if upper is not None else hi) + pad


def plot_single_or_multi_val(
    val: Union[Tensor, Sequence[Tensor], Dict[str, Tensor], Sequence[Dict[str, Tensor]]],
    ax: Optional[_AX_TYPE] = None,
    higher_is_better: Optional[bool] = None,
    lower_bound: Optional[float] = None,
    upper_bound: Optional[float] = None,
    legend_name: Optional[str] = None,
    name: Optional[str] = None,
) -> _PLOT_OUT_TYPE:
    """Plot one value, a per-class vector, a dict of values, or a history of any of those."""
    plt = _pyplot()
    series, steps = _series_of(val, legend_name)
    fig, ax = plt.subplots() if ax is None else (None, ax)
    for s in series:
        ax.plot(s.x, s.y, linestyle="-" if s.line else "None", label=s.label, **_MARKER)
    ax.get_xaxis().set_visible(steps > 0)
    if steps:
        ax.set_xlabel("Step")
        ax.set_xticks(np.arange(steps))
    handles, labels = ax.get_legend_handles_labels()
    if handles and labels:
        ax.legend(handles, labels, loc="upper center", bbox_to_anchor=(0.5, 1.15), ncol=3, fancybox=True, shadow=True)
    bottom, top = _padded_limits(*ax.get_ylim(), lower_bound, upper_bound)
    ax.set_ylim(bottom=bottom, top=top)
    ax.grid(True)
    ax.set_ylabel(name)
    left, right = ax.get_xlim()
    bounds = [b for b in (lower_bound, upper_bound) if b is not None]
    ax.hlines(bounds, left, right, linestyles="dashed", colors="k")
    optimum = {True: upper_bound, False: lower_bound}.get(higher_is_better) if higher_is_better is not None else None
    if optimum is not None:  # make room left of the data and label the optimal bound
        ax.set_xlim(left - 0.1 * (right - left), right)
        ax.text(left, optimum, s="Optimal \n value", horizontalalignment="center", verticalalignment="center")
    return fig, ax


def _get_col_row_split(n: int) -> Tuple[int, int]:
    """(rows, cols) of the most square grid with at least ``n`` cells."""
    side = sqrt(n)
    if int(side) ** 2 == n:
        return int(side), int(side)
    if floor(side) * ceil(side) >= n:
        return floor(side), ceil(side)
    return ceil(side), ceil(side)


def trim_axs(axs: Any, nb: int) -> Any:
    """Remove the unused axes of a subplot grid and return the first ``nb``."""
    if not isinstance(axs, np.ndarray):
        return axs
    for extra in axs.flat[nb:]:
        extra.remove()
    return axs.flat[:nb]


class _Panel(NamedTuple):
    title: Optional[str]
    matrix: np.ndarray
    ticks: List[Any]


def _confmat_panels(confmat: Tensor, labels: Optional[List[Union[int, str]]]) -> List[_Panel]:
    """One panel per label for a multilabel ``[L, 2, 2]`` stack, one panel for a ``[C, C]`` matrix."""
    if confmat.ndim == 3:
        names = labels if labels is not None else list(range(confmat.shape[0]))
        return [_Panel(f"Label {names[i]}", _host(confmat[i]), ["0", "1"]) for i in range(confmat.shape[0])]
    n = confmat.shape[0]
    if labels is not None and len(labels) != n:
        raise ValueError(
            "Expected number of elements in arg `labels` to match number of labels in confmat but "
            f"got {len(labels)} and {n}"
        )
    return [_Panel(None, _host(confmat), list(labels) if labels is not None else list(range(n)))]


def plot_confusion_matrix(
    confmat: Tensor,
    ax: Optional[_AX_TYPE] = None,
    add_text: bool = True,
    labels: Optional[List[Union[int, str]]] = None,
    cmap: Optional[Any] = None,
) -> _PLOT_OUT_TYPE:
    """Heat map of a ``[C, C]`` confusion matrix (or a grid of ``[2, 2]`` ones for a multilabel ``[L, 2, 2]``)."""
    plt = _pyplot()
    panels = _confmat_panels(confmat, labels)
    rows, cols = _get_col_row_split(len(panels)) if confmat.ndim == 3 else (1, 1)
    fig, axs = plt.subplots(nrows=rows, ncols=cols) if ax is None else (ax.get_figure(), ax)
    axs = trim_axs(axs, len(panels))
    for i, panel in enumerate(panels):
        a = axs[i] if (rows != 1 and cols != 1) else axs
        if panel.title is not None:
            a.set_title(panel.title, fontsize=15)
        a.imshow(panel.matrix, cmap=cmap)
        a.set_xlabel("Predicted class", fontsize=15)
        a.set_ylabel("True class", fontsize=15)
        k = len(panel.ticks)
        a.set_xticks(list(range(k)))
        a.set_yticks(list(range(k)))
        a.set_xticklabels(panel.ticks, rotation=45, fontsize=10)
        a.set_yticklabels(panel.ticks, rotation=25, fontsize=10)
        if add_text:
            for r, c in product(range(k), range(k)):
                a.text(c, r, str(round(float(panel.matrix[r, c]), 2)), ha="center", va="center", fontsize=15)
    return fig, axs


def _curve_series(curve: Sequence[Any], score: Optional[Tensor], legend_name: Optional[str]) -> List[_Series]:
    """(x, y[, thresholds]) of one curve or of per-class curves -> series labelled with their AUC when given."""
    if len(curve) < 2:
        raise ValueError(f"Expected 2 or 3 elements in curve but got {len(curve)}")
    if score is not None and not isinstance(score, Tensor):
        raise ValueError(f"Expected score to be a tensor but got {type(score)}")
    x, y = curve[0], curve[1]
    if isinstance(x, Tensor) and isinstance(y, Tensor) and x.ndim == 1 and y.ndim == 1:
        return [_Series(f"AUC={score.item():0.3f}" if score is not None else None, _host(x), _host(y), True)]
    per_class = (isinstance(x, list) and isinstance(y, list)) or (
        isinstance(x, Tensor) and isinstance(y, Tensor) and x.ndim == 2 and y.ndim == 2)
    if not per_class:
        raise ValueError(
            f"Unknown format for argument `x` and `y`. Expected either list or tensors but got {type(x)} and {type(y)}."
        )
    out = []
    for i, (xi, yi) in enumerate(zip(x, y)):
        label = f"{legend_name}_{i}" if legend_name is not None else str(i)
        if score is not None:
            label += f" AUC={score[i].item():0.3f}"
        out.append(_Series(label, _host(xi), _host(yi), True))
    return out


def plot_curve(
    curve: Union[Tuple[Tensor, Tensor, Tensor], Tuple[Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]],
    score: Optional[Tensor] = None,
    ax: Optional[_AX_TYPE] = None,
    label_names: Optional[Tuple[str, str]] = None,
    legend_name: Optional[str] = None,
    name: Optional[str] = None,
) -> _PLOT_OUT_TYPE:
    """ROC / PR style curve(s), each labelled with its score when one is given."""
    plt = _pyplot()
    series = _curve_series(curve, score, legend_name)
    fig, ax = plt.subplots() if ax is None else (None, ax)
    for s in series:
        ax.plot(s.x, s.y, linestyle="-", linewidth=2, label=s.label)
    single = len(series) == 1 and isinstance(curve[0], Tensor) and curve[0].ndim == 1
    if single and label_names is not None:
        ax.set_xlabel(label_names[0])
        ax.set_ylabel(label_names[1])
    if any(s.label is not None for s in series):
        ax.legend()
    ax.grid(True)
    ax.set_title(name)
    return fig, ax
