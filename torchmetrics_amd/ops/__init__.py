"""Device-dispatching entry points for the hand-written HIP kernels (``csrc/`` -> ``_C/libtm_amd.so``).

Every op has exactly two implementations, selected by the *device of its inputs* (not by availability):

* ROCm tensors (``tensor.is_cuda``) -> ``torch.ops.tm_amd.*`` HIP kernels for gfx950.  If the library is missing
  on a GPU host the call raises: there is no silent eager fallback on the GPU.
  The per-batch hot ops (``mc_update``, ``bin_update``, ``moments_update``, the stat-score finalizers and
  ``stat_reduce``) enter the same C++ launchers through ``_C/_fastcall.so`` (``csrc/bindings/fastcall.cpp``), a
  METH_FASTCALL CPython module that skips the boxed dispatcher call (~5.5 us -> ~1.5 us of host time per update).
* CPU tensors -> the host implementation in :mod:`torchmetrics_amd.ops._cpu` (ATen ops), which is the CPU
  device implementation of the same contract (used by CPU/gloo runs and as the numerics oracle in tests).
"""
import os
import struct
import threading
from pathlib import Path
from typing import Any, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_amd.ops import _cpu

_LIB_PATH = Path(__file__).resolve().parent.parent / "_C" / "libtm_amd.so"
_FAST_PATH = _LIB_PATH.parent / "_fastcall.so"
_lock = threading.Lock()
_state = {"loaded": False, "error": None, "fast_error": None}
_fast_mod = None  # the _fastcall extension module once loaded (or a torch.ops shim if it could not be)


class _DispatcherShim:
    """``_fastcall`` stand-in routing through ``torch.ops.tm_amd`` (used only if ``_fastcall.so`` failed to load)."""

    def __getattr__(self, name):
        op = getattr(torch.ops.tm_amd, name)
        if name in ("mc_update", "bin_update", "moments_update", "stat_reduce"):
            ncontig = 4 if name == "stat_reduce" else 2

            def call(*args, _op=op, _n=ncontig):
                return _op(*[a.contiguous() for a in args[:_n]], *args[_n:])

            return call
        return op


def _load_fastcall() -> None:
    global _fast_mod
    import importlib.util

    try:
        spec = importlib.util.spec_from_file_location("_fastcall", _FAST_PATH)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _fast_mod = mod
        from torchmetrics_amd.utils import profiling

        if profiling.ENABLED:
            mod.set_ranges(True)
    except Exception as err:  # noqa: BLE001 - the dispatcher path is the same native code, just slower to enter
        _state["fast_error"] = err
        _fast_mod = _DispatcherShim()


def _fast():
    if _fast_mod is None:
        load_native(strict=True)
    return _fast_mod


def native_updater(kind: str, state: dict, fallback: Any, *extra: Any) -> Any:
    """A native ``update`` callable bound to a metric's ``__dict__`` (``csrc/bindings/fastcall.cpp``), or ``None``
    where it does not apply (no GPU, native library missing, ``TORCHMETRICS_AMD_STRICT=1``).  Inputs off its fast path
    go to ``fallback`` (the metric's Python update)."""
    from torchmetrics_amd.utils import validation

    if validation.STRICT or not torch.cuda.is_available() or not load_native(strict=False):
        return None
    mod = _fast_mod
    factory = getattr(mod, f"{kind}_updater", None) if not isinstance(mod, _DispatcherShim) else None
    if factory is None:
        return None
    fn = factory(*extra, state, fallback) if extra else factory(state, fallback)
    fn.range_name = f"tm.update/{_owner_name(fallback)}"  # roctx range of the native call (utils/profiling.py)
    return fn


def _owner_name(fallback: Any) -> str:
    """Class name of the metric a bound ``update`` / ``forward`` (or its ``functools.wraps`` wrapper) belongs to."""
    owner = getattr(getattr(fallback, "__wrapped__", fallback), "__self__", None)
    return type(owner).__name__ if owner is not None else "Metric"


FWD_CONFMAT, FWD_MULTICLASS, FWD_BINARY, FWD_MULTILABEL = 0, 1, 2, 3
STAT_KINDS = {"accuracy": 0, "hamming": 1, "precision": 2, "recall": 3, "specificity": 4, "fbeta": 5}


def native_forward(kind: int, state: dict, fallback: Any, stat_kind: str = "accuracy") -> Any:
    """A native ``forward`` callable bound to a metric's ``__dict__`` (``csrc/bindings/fastcall.cpp`` ``NativeForward``)
    or ``None`` where it does not apply (no GPU, native library missing, ``TORCHMETRICS_AMD_STRICT=1``,
    ``TORCHMETRICS_AMD_NATIVE_FORWARD=0``).  Calls off its fast path go to ``fallback`` (``Metric.forward``)."""
    from torchmetrics_amd.utils import validation

    if (validation.STRICT or os.environ.get("TORCHMETRICS_AMD_NATIVE_FORWARD", "1") == "0"
            or not torch.cuda.is_available() or not load_native(strict=False)):
        return None
    mod = _fast_mod
    factory = getattr(mod, "forward_native", None) if not isinstance(mod, _DispatcherShim) else None
    if factory is None:
        return None
    fn = factory(kind, state, fallback, STAT_KINDS[stat_kind])
    fn.range_name = f"tm.forward/{_owner_name(fallback)}"
    return fn


def read_word(word: Tensor) -> int:
    """The int32 word ``word[0]``: on ROCm through mapped host memory + a stream sync (``read_word_sync``: the stream is
    then known idle, so the caller's next ``torch.cuda.synchronize()`` costs nothing), else ``.item()``."""
    if word.is_cuda and word.dtype == torch.int32:
        mod = _fast_mod if _fast_mod is not None else (_fast() if native_available() else None)
        fn = getattr(mod, "read_word", None) if mod is not None else None
        if fn is not None:
            return fn(word)
    return int(word.reshape(-1)[0].item())


READ_WORDS_SPIN_US = 2000  # how long read_words spins before a blocking stream sync (a busy queue ahead of it)


def read_words(table: Tensor, anchor: Tensor) -> Optional[List[int]]:
    """Every word of ``table`` (CPU int64 ``[n <= 128, 2]`` rows of (device pointer, code), see
    ``csrc/common/compute_tasks.hip`` read_words) through one gather kernel into mapped host memory and a spin on the
    sequence number it stores after them; None without the native module (the caller takes the gather + sync)."""
    mod = _fast_mod if _fast_mod is not None else (_fast() if native_available() else None)
    fn = getattr(mod, "read_words", None) if mod is not None else None
    if fn is None or not anchor.is_cuda:
        return None
    return fn(table, anchor, READ_WORDS_SPIN_US)


def sole_ref(d: dict, key: Any) -> bool:
    """Whether ``d[key]`` is a tensor whose Python object is referenced by ``d`` alone (``_sole_ref`` in
    ``csrc/bindings/fastcall.cpp``: the exact strong-reference count, read from C).  Without the native module:
    False (callers then take their always-correct out-of-place path)."""
    mod = _fast_mod
    if mod is None:
        if not native_available():
            return False
        mod = _fast()
    fn = getattr(mod, "_sole_ref", None)
    return bool(fn(d, key)) if fn is not None else False


def native_library_path() -> Path:
    return _LIB_PATH


def load_native(strict: bool = True) -> bool:
    """Load ``libtm_amd.so`` (idempotent). With ``strict`` a missing/broken library raises."""
    if _state["loaded"]:
        return True
    with _lock:
        if _state["loaded"]:
            return True
        try:
            if not _LIB_PATH.exists():
                raise FileNotFoundError(
                    f"{_LIB_PATH} not found: build the HIP kernels with `python tools/build_ext.py` "
                    "(or `python -c 'import __graft_entry__ as g; g.build()'`)"
                )
            torch.ops.load_library(str(_LIB_PATH))
            _load_fastcall()
            _state["loaded"] = True
        except Exception as err:  # noqa: BLE001
            _state["error"] = err
            if strict:
                raise RuntimeError(f"torchmetrics_amd native HIP library unavailable: {err}") from err
            return False
    return True


def native_available() -> bool:
    return load_native(strict=False)


def _ops():
    load_native(strict=True)
    return torch.ops.tm_amd


# ------------------------------------------------------------------------------------------------ classification
MC_CONFMAT = 0
MC_STATS = 1


def mc_update(
    preds: Tensor,
    target: Tensor,
    out: Tensor,
    flag: Tensor,
    num_classes: int,
    ignore_index: Optional[int],
    mode: int,
    samplewise: bool = False,
) -> None:
    """Multiclass histogram update (see ``csrc/classification/stat_scores.hip``).

    ``preds``: float scores ``[N, C, ...]`` (argmax) or int labels ``[N, K, ...]``; ``target``: ``[N, ...]``.
    ``mode=MC_CONFMAT`` accumulates ``out[C, C]``; ``mode=MC_STATS`` accumulates the ``[G, 3C+1]`` workspace.
    """
    if preds.is_cuda:
        (_fast_mod or _fast()).mc_update(
            preds, target, out, flag, num_classes, 0 if ignore_index is None else ignore_index,
            ignore_index is not None, mode, samplewise,
        )
    else:
        _cpu.mc_update(preds, target, out, flag, num_classes, ignore_index, mode, samplewise)


def mc_bootstrap_update(preds: Tensor, target: Tensor, weights: Tensor, ws: Tensor, flag: Tensor, num_classes: int,
                        ignore_index: Optional[int]) -> None:
    """Weighted multiclass stat workspace for B bootstraps at once (``csrc/classification/bootstrap.hip``):
    ``weights`` int32 ``[N, B]`` sample multiplicities; ``ws`` int64 ``[B, 3C + 1]`` (fold with
    :func:`mc_stats_finalize`)."""
    if preds.is_cuda:
        _ops().mc_bootstrap_update(preds, target, weights, ws, flag, int(num_classes),
                                   0 if ignore_index is None else int(ignore_index), ignore_index is not None)
    else:
        _cpu.mc_bootstrap_update(preds, target, weights, ws, flag, num_classes, ignore_index)


def mc_stats_finalize(ws: Tensor, num_classes: int, micro: bool, accumulate: bool, tp: Tensor, fp: Tensor,
                      tn: Tensor, fn: Tensor) -> None:
    if ws.is_cuda:
        (_fast_mod or _fast()).mc_stats_finalize(ws, num_classes, micro, accumulate, tp, fp, tn, fn)
    else:
        _cpu.mc_stats_finalize(ws, num_classes, micro, accumulate, tp, fp, tn, fn)


def bin_update(preds: Tensor, target: Tensor, ws: Tensor, flag: Tensor, not_prob: Tensor, num_labels: int,
               threshold: float, ignore_index: Optional[int], samplewise: bool = False,
               prob_check_all: bool = True) -> None:
    """Binary / multilabel tp/fp/fn/count update for ``[N, L, ...]`` inputs into a ``[G, 7]`` workspace.  On ROCm
    the per-block partial rows may be left pending for ``bin_stats_finalize`` / ``bin_confmat_finalize`` (one fused
    fold + finalize launch): read ``ws`` itself only after :func:`bin_flush`.

    ``prob_check_all=False`` excludes ignored positions from the logits-vs-probabilities decision.
    """
    if preds.is_cuda:
        (_fast_mod or _fast()).bin_update(
            preds, target, ws, flag, not_prob, num_labels, float(threshold),
            0 if ignore_index is None else ignore_index, ignore_index is not None, samplewise, prob_check_all,
        )
    else:
        _cpu.bin_update(preds, target, ws, flag, not_prob, num_labels, threshold, ignore_index, samplewise,
                        prob_check_all)


def bin_flush(ws: Tensor) -> None:
    """Fold the per-block rows a ROCm ``bin_update`` left pending for its finalizer into ``ws`` (for readers of the
    raw workspace; the two finalizers fold and finalize in one launch themselves)."""
    if ws.is_cuda:
        _ops().bin_flush_pending(ws)


def bin_confmat_finalize(ws: Tensor, not_prob: Tensor, confmat: Tensor) -> None:
    """Fold a ``[G, 7]`` workspace into ``[G, 2, 2]`` confusion matrices (in place) and re-zero it."""
    if ws.is_cuda:
        (_fast_mod or _fast()).bin_confmat_finalize(ws, not_prob, confmat)
    else:
        _cpu.bin_confmat_finalize(ws, not_prob, confmat)


def bin_stats_finalize(ws: Tensor, not_prob: Tensor, accumulate: bool, tp: Tensor, fp: Tensor, tn: Tensor,
                       fn: Tensor) -> None:
    if ws.is_cuda:
        (_fast_mod or _fast()).bin_stats_finalize(ws, not_prob, accumulate, tp, fp, tn, fn)
    else:
        _cpu.bin_stats_finalize(ws, not_prob, accumulate, tp, fp, tn, fn)


def histogram(x: Tensor, minlength: int) -> Tensor:
    """Deterministic integer bincount (int64 counts)."""
    if x.is_cuda:
        out = torch.zeros(int(minlength), dtype=torch.int64, device=x.device)
        flag = torch.zeros(1, dtype=torch.int32, device=x.device)
        x = x if x.dtype in (torch.int64, torch.int32, torch.uint8) else x.long()
        _ops().histogram(x.contiguous(), out, flag)
        return out
    x = x.long()
    ok = (x >= 0) & (x < minlength)
    if not bool(ok.all()):  # out-of-range keys are skipped, as in the kernel
        x = x[ok]
    return torch.bincount(x, minlength=minlength)


# ------------------------------------------------------------------------------- windowed image statistics
_BOX_MAX_WINDOW = 32


def box_rmse_maps(preds: Tensor, target: Tensor, window: int, want_target: bool) -> Optional[Tuple[Tensor, Tensor]]:
    """Batch-summed ``sqrt(box_mean((t - p)^2))`` map ``[C, H, W]`` and (``want_target``) ``box_mean(t) / w^2`` map,
    with the reference's symmetric padding (``csrc/image/window_stats.hip``); ``None`` where the kernel does not
    apply (CPU, window > 32 or larger than the image)."""
    if not preds.is_cuda or window > _BOX_MAX_WINDOW or window > preds.shape[2] or window > preds.shape[3]:
        return None
    c, h, w = preds.shape[1:]
    rmse_map = torch.empty(c, h, w, dtype=preds.dtype, device=preds.device)
    t_map = torch.empty(c, h, w, dtype=preds.dtype, device=preds.device) if want_target else \
        torch.empty(0, dtype=preds.dtype, device=preds.device)
    _ops().box_rmse_maps(preds.contiguous(), target.contiguous(), int(window), rmse_map, t_map)
    return rmse_map, t_map


INFO_MEASURE_IDS = {"kl_divergence": 0, "alpha_divergence": 1, "beta_divergence": 2, "ab_divergence": 3,
                    "renyi_divergence": 4, "l1_distance": 5, "l2_distance": 6, "l_infinity_distance": 7,
                    "fisher_rao_distance": 8}


def info_measure(p: Tensor, t: Tensor, measure: str, alpha: float, beta: float) -> Optional[Tensor]:
    """InfoLM information measure per row of fp32 ``[N, V]`` distributions in one launch (``csrc/text/infolm.hip``),
    including the reference's ``nan_to_num``; ``None`` off-GPU / non-fp32 / autograd."""
    if not _no_grad_path(p, t) or p.dtype != torch.float32 or t.dtype != torch.float32 or p.dim() != 2 \
            or p.shape != t.shape:
        return None
    out = torch.empty(p.shape[0], dtype=torch.float32, device=p.device)
    mid = INFO_MEASURE_IDS[measure]
    _ops().info_measure(p.contiguous(), t.contiguous(), mid, float(1.0 if mid == 2 else alpha), float(beta), out)
    return out


def infolm_accumulate(logits: Tensor, temperature: float, w: Tensor, rows: Tensor, acc: Tensor) -> None:
    """``acc[rows[r]] += w[r] * softmax(logits[r] / temperature)`` for masked-LM logits ``[R, V]`` whose ``rows`` (CPU
    int64, non-decreasing: one sentence's positions are consecutive) name the destination row of ``acc`` fp32 [N, V];
    two launches, no [R, V] probabilities (``csrc/text/infolm.hip``)."""
    if rows.numel() == 0:
        return
    sents, counts = torch.unique_consecutive(rows, return_counts=True)
    seg = torch.zeros(counts.numel() + 1, dtype=torch.int64)
    torch.cumsum(counts, 0, out=seg[1:])
    dev = logits.device
    _ops().infolm_accumulate(logits.contiguous(), float(temperature), w.to(dev, torch.float32).contiguous(),
                             seg.to(dev), sents.to(dev, torch.int64), acc)


def nominal_table_stats(cm: Tensor) -> Optional[Tensor]:
    """fp64 ``[B, 8]`` statistics of int64 contingency tables ``[B, K, K]`` (``csrc/nominal/table_stats.hip``: n, r, c,
    chi^2, Yates chi^2, sum p_xy log(p_y / p_xy), H(X)); ``None`` off-GPU or for K > 1024."""
    if not cm.is_cuda or cm.dim() != 3 or cm.shape[1] != cm.shape[2] or cm.shape[1] > 1024 or cm.shape[1] < 1:
        return None
    out = torch.empty(cm.shape[0], 8, dtype=torch.float64, device=cm.device)
    _ops().nominal_table_stats(cm.to(torch.int64).contiguous(), out)
    return out


def _no_grad_path(*ts: Tensor) -> bool:
    """ROCm tensors that autograd does not need to see through (the kernels are forward-only)."""
    return ts[0].is_cuda and not (torch.is_grad_enabled() and any(t.requires_grad for t in ts))


def sam_angles(preds: Tensor, target: Tensor, want_map: bool, want_sum: bool) -> Optional[Tuple[Optional[Tensor],
                                                                                                Optional[Tensor]]]:
    """Spectral angles of ``[B, C, H, W]`` images (``csrc/image/spectral.hip``): the ``[B, H, W]`` angle map and/or
    their fp64 sum (0-d), one pass; ``None`` off-GPU or when autograd needs the graph."""
    if not _no_grad_path(preds, target):
        return None
    p, t = preds.contiguous(), target.contiguous()
    b, _, h, w = p.shape
    amap = torch.empty(b, h, w, dtype=p.dtype, device=p.device) if want_map else p.new_empty(0)
    blocks = max(1, min((b * h * w + 255) // 256, 2048))
    part = torch.empty(blocks, dtype=torch.float64, device=p.device) if want_sum else \
        torch.empty(0, dtype=torch.float64, device=p.device)
    _ops().sam_angles(p, t, amap, part)
    return (amap if want_map else None), (part.sum() if want_sum else None)


def band_stats(preds: Tensor, target: Tensor) -> Optional[Tensor]:
    """Per (image, band) of ``[B, C, H, W]`` images: fp64 ``[B, C, 2]`` = (Σ(p - t)², Σt) in one pass
    (``csrc/image/spectral.hip``); ``None`` off-GPU or when autograd needs the graph."""
    if not _no_grad_path(preds, target):
        return None
    b, c = preds.shape[:2]
    p, t = preds.contiguous().reshape(b * c, -1), target.contiguous().reshape(b * c, -1)
    bpr = max(1, min(64, p.shape[1] // (256 * 32)))
    part = torch.empty(b * c, bpr, 2, dtype=torch.float64, device=p.device)
    _ops().band_stats(p, t, part)
    return part.sum(1).view(b, c, 2)


def neighbour_diff_stats(x: Tensor, y: Optional[Tensor], block_size: int, squared: bool) -> Optional[Tensor]:
    """Per image f64 ``[B, 5]``: ``Σ(x - y)^2``, neighbour differences across / off ``block_size`` boundaries
    (horizontal, then vertical); ``None`` off-GPU."""
    if not x.is_cuda:
        return None
    out = torch.empty(x.shape[0], 5, dtype=torch.float64, device=x.device)
    yy = y.contiguous() if y is not None else torch.empty(0, dtype=x.dtype, device=x.device)
    _ops().neighbour_diff_stats(x.contiguous(), yy, int(block_size), bool(squared), out)
    return out


# ----------------------------------------------------------------------------------- clustering / nominal
_DENSE_CONTINGENCY_MAX = 1 << 26  # dense-range bins before falling back to unique() relabelling


def _label_ranges(*xs: Tensor) -> List[Tuple[int, int]]:
    """``[(min, max)]`` of integer label tensors: one ``label_minmax`` launch pair each, ONE host read for all."""
    mm = torch.cat([_ops().label_minmax(x.contiguous()) for x in xs]).tolist()
    return [(mm[2 * i], mm[2 * i + 1]) for i in range(len(xs))]


def contingency(preds: Tensor, target: Tensor) -> Tensor:
    """``[n_target_values, n_pred_values]`` co-occurrence counts over the sorted distinct values of each.

    ROCm, integer labels: one min/max pass per tensor (one host read), then the 2-D histogram over the dense label
    ranges with the key built in registers (``csrc/clustering/cluster.hip``); value ranges that never occur are
    dropped by their zero marginals, which leaves exactly the sorted-unique rows / columns.  Otherwise (CPU, float
    labels, huge ranges): ``unique(return_inverse)`` relabelling + the histogram kernel."""
    if preds.is_cuda and not preds.is_floating_point() and not target.is_floating_point() and preds.numel():
        (tmin, tmax), (pmin, pmax) = _label_ranges(target, preds)
        rt, rp = tmax - tmin + 1, pmax - pmin + 1
        if rt * rp <= _DENSE_CONTINGENCY_MAX:
            p = preds if preds.dtype in (torch.int64, torch.int32, torch.uint8) else preds.long()
            t = target if target.dtype in (torch.int64, torch.int32, torch.uint8) else target.long()
            cont = torch.zeros(rt, rp, dtype=torch.int64, device=preds.device)
            _ops().contingency_dense(t.contiguous(), p.contiguous(), tmin, pmin, cont)
            rows, cols = cont.sum(1) > 0, cont.sum(0) > 0
            if bool(rows.all()) and bool(cols.all()):
                return cont
            return cont[rows][:, cols]
    p_cls, p_idx = torch.unique(preds, return_inverse=True)
    t_cls, t_idx = torch.unique(target, return_inverse=True)
    kp, kt = p_cls.numel(), t_cls.numel()
    return histogram(t_idx * kp + p_idx, kt * kp).reshape(kt, kp)


def dense_labels(labels: Tensor) -> Tuple[Tensor, int]:
    """``(ids, K)``: ``labels`` relabelled to ``0..K-1`` in sorted-value order (``unique(return_inverse)``).  ROCm
    integer labels with a modest range: a presence histogram over the range and a prefix sum, no sort."""
    if labels.is_cuda and not labels.is_floating_point() and labels.numel():
        ((lo, hi),) = _label_ranges(labels)
        r = hi - lo + 1
        if r <= _DENSE_CONTINGENCY_MAX:
            shifted = labels.long() - lo
            present = histogram(shifted, r) > 0
            remap = torch.cumsum(present, 0) - 1
            return remap[shifted], int(present.sum())
    uniq, inv = torch.unique(labels, return_inverse=True)
    return inv, uniq.numel()


def cluster_sums(data: Tensor, ids: Tensor, k: int) -> Tuple[Tensor, Tensor]:
    """Per-cluster feature sums (fp64 ``[K, D]``) and sizes (int64 ``[K]``) for dense ids."""
    if data.is_cuda:
        sums = torch.zeros(k, data.shape[1], dtype=torch.float64, device=data.device)
        sizes = torch.zeros(k, dtype=torch.int64, device=data.device)
        _ops().cluster_sums(data.contiguous(), ids.contiguous(), k, sums, sizes)
        return sums, sizes
    sums = torch.zeros(k, data.shape[1], dtype=torch.float64).index_add_(0, ids, data.double())
    return sums, torch.bincount(ids, minlength=k)


def cluster_dispersion(data: Tensor, ids: Tensor, centroids: Tensor, p: float = 2.0) -> Tuple[Tensor, Tensor, Tensor]:
    """Per cluster Σ ||x - c||_p and max ||x - c||_p (fp64 ``[K]``), and the total Σ ||x - c||² (fp64 scalar)."""
    k = centroids.shape[0]
    cent = centroids.to(torch.float64).contiguous()
    if data.is_cuda and (k * data.shape[1] + 2 * k) * 8 <= 64 * 1024:
        dsum = torch.zeros(k, dtype=torch.float64, device=data.device)
        dmax = torch.zeros(k, dtype=torch.float64, device=data.device)
        sq = torch.zeros(1, dtype=torch.float64, device=data.device)
        _ops().cluster_dispersion(data.contiguous(), ids.contiguous(), cent, float(p), dsum, dmax, sq)
        return dsum, dmax, sq[0]
    diff = data.double() - cent[ids]
    dist = torch.linalg.vector_norm(diff, ord=p, dim=1)
    dsum = torch.zeros(k, dtype=torch.float64, device=data.device).index_add_(0, ids, dist)
    dmax = torch.zeros(k, dtype=torch.float64, device=data.device).scatter_reduce(0, ids, dist, reduce="amax")
    return dsum, dmax, (diff * diff).sum()


# ------------------------------------------------------------------------------------- sorted curves / ranks
CLF_T_BINARY = 0  # target[e] == pos_label, one segment
CLF_T_OVR = 1  # target[e] == segment index (multiclass one-vs-rest columns)
CLF_T_ELEM = 2  # target stored like the scores (multilabel columns, label-ranking rows)
EMIT_CURVE = 1
EMIT_RANKS = 2


def clf_curve(scores: Tensor, target: Tensor, S: int, M: int, seg_stride: int, elem_stride: int, tmode: int,
              pos_label: int = 1, ignore_index: Optional[int] = None, weights: Optional[Tensor] = None,
              emit: int = 0) -> list:
    """Segmented descending sort + tie-run scan over ``S`` segments of ``M`` scores (``csrc/sort/clf_curve.hip``).

    Element ``e`` of segment ``s`` is ``scores[s * seg_stride + e * elem_stride]`` (element strides of ``scores``
    itself).  Returns ``[stats [S, 8] fp64 = (P, N, auroc_area, ap_sum, coverage, 0, n_runs, 0), fps, tps, thr, ranks]``
    (curve tensors ``[S, M]`` compacted per segment, present with ``emit & EMIT_CURVE``; ``ranks`` average 1-based
    ranks by flat id ``s * M + e`` with ``emit & EMIT_RANKS``).
    """
    if scores.is_cuda:
        w = None if weights is None else weights.to(torch.float64).contiguous()
        return list(_ops().clf_curve(scores, target, w, S, M, seg_stride, elem_stride, tmode, pos_label,
                                     0 if ignore_index is None else ignore_index, ignore_index is not None, emit))
    return _cpu.clf_curve(scores, target, weights, S, M, seg_stride, elem_stride, tmode, pos_label, ignore_index,
                          emit)


RETRIEVAL_KIND = {name: i for i, name in enumerate(_cpu.RETRIEVAL_KINDS)}


def retrieval_metric(preds: Tensor, target: Tensor, indexes: Tensor, kind: str, top_k: Optional[int] = None,
                     adaptive_k: bool = False) -> list:
    """Per-query retrieval metric for all queries at once (``csrc/sort/retrieval.hip``).

    Returns ``[values fp64 [n], empty uint8 [n], n_queries int32 [1]]``; the first ``n_queries`` entries are the
    queries in ascending id order.  ``empty`` marks queries without relevant documents (fall-out: without
    non-relevant ones).  Nothing is read back to the host.
    """
    k = RETRIEVAL_KIND[kind]
    tk = -1 if top_k is None else int(top_k)
    if preds.is_cuda:
        t = target if target.dtype != torch.bool else target.to(torch.uint8)
        return list(_ops().retrieval_metric(preds.reshape(-1).contiguous(), t.reshape(-1).contiguous(),
                                            indexes.reshape(-1).contiguous(), k, tk, adaptive_k))
    return _cpu.retrieval_metric(preds.reshape(-1), target.reshape(-1), indexes.reshape(-1), k, tk, adaptive_k)


def retrieval_pr_curve(preds: Tensor, target: Tensor, indexes: Tensor, max_k: Optional[int] = None,
                       adaptive_k: bool = False) -> list:
    """Precision@k / recall@k curves (k = 1..K) of every query (``csrc/sort/retrieval.hip``).

    Returns ``[precision f32 [n_queries, K], recall f32 [n_queries, K], empty uint8 [n_queries]]``, queries in
    ascending id order; ``K = max_k`` or the largest query size.  One host read (the query count and largest size,
    which fix the output shape).
    """
    mk = -1 if max_k is None else int(max_k)
    if preds.is_cuda:
        t = target if target.dtype != torch.bool else target.to(torch.uint8)
        return list(_ops().retrieval_pr_curve(preds.reshape(-1).contiguous(), t.reshape(-1).contiguous(),
                                              indexes.reshape(-1).contiguous(), mk, adaptive_k))
    return _cpu.retrieval_pr_curve(preds.reshape(-1), target.reshape(-1), indexes.reshape(-1), mk, adaptive_k)


def paired_cosine(a: Tensor, b: Tensor, scale: float = 1.0) -> Tensor:
    """``scale * cos(a_i, b_i)`` of ``[N, D]`` embedding pairs as fp32 ``[N]`` (``csrc/multimodal/clip.hip``: one wave
    per pair, no normalised copies)."""
    if a.is_cuda:
        if b.dtype != a.dtype:
            b = b.to(a.dtype)
        return _ops().paired_cosine(a.contiguous(), b.contiguous(), float(scale))
    return _cpu.paired_cosine(a, b, scale)


def prompt_pair_prob(img: Tensor, anchors: Tensor, scale: float = 100.0) -> Tensor:
    """Softmax of ``scale * img @ anchors^T`` over each (positive, negative) anchor pair -> probability of the
    positive prompt, fp32 ``[N, P]`` (``csrc/multimodal/clip.hip``)."""
    # the kernel stages 32 anchors x D in <= 128 KB of LDS (D <= 1024 in fp32; CLIP's projection dims are 512-1024)
    if img.is_cuda and 32 * img.shape[-1] * (8 if img.dtype == torch.float64 else 4) <= 128 * 1024:
        if anchors.dtype != img.dtype:
            anchors = anchors.to(img.dtype)
        return _ops().prompt_pair_prob(img.contiguous(), anchors.contiguous(), float(scale))
    return _cpu.prompt_pair_prob(img, anchors, scale)


def kendall_stats(x: Tensor, y: Tensor) -> Tensor:
    """Per column of ``[n, k]`` inputs: ``[disc, tx, tx1, tx2, ty, ty1, ty2, txy, ux, uy]`` (fp64) -- discordant
    pairs, tie terms of x / y (sum of t(t-1)/2, t(t-1)(t-2), t(t-1)(2t+5)), joint ties and distinct counts
    (``csrc/sort/kendall.hip``: radix sorts + merge-path inversion count, O(n log n))."""
    if x.is_cuda:
        if y.dtype != x.dtype:
            y = y.to(x.dtype)
        if not x.is_floating_point():
            x, y = x.double(), y.double()
        return _ops().kendall_stats(x, y)
    return _cpu.kendall_stats(x, y)


class CalibrationWorkspace:
    """Per-metric device scratch of :func:`mc_calibration_update` (candidate rows + double-buffered decision word)."""

    __slots__ = ("cand", "notprob", "slot")

    def __init__(self) -> None:
        self.cand: Optional[Tensor] = None
        self.notprob: Optional[Tensor] = None
        self.slot = 0


_EMPTY_FLAG: dict = {}


def mc_calibration_update(preds: Tensor, target: Tensor, ws: CalibrationWorkspace,
                          flag: Optional[Tensor] = None) -> "tuple[Tensor, Tensor]":
    """Top-label ``(confidences, accuracies)`` of ``[M, C]`` ROCm scores (softmax applied iff any score of the batch
    is outside [0, 1]) in two launches (``csrc/classification/calibration.hip``); target range errors go to
    ``flag``."""
    m = preds.shape[0]
    dev = preds.device
    if ws.cand is None or ws.cand.device != dev or ws.cand.numel() < 4 * m:
        ws.cand = torch.empty(max(4 * m, 1024), dtype=torch.float32, device=dev)
        ws.notprob = torch.zeros(2, dtype=torch.int32, device=dev)
        ws.slot = 0
    conf = torch.empty(m, dtype=torch.float32, device=dev)
    acc = torch.empty(m, dtype=torch.float32, device=dev)
    if flag is None:
        key = (dev.type, dev.index)
        flag = _EMPTY_FLAG.get(key)
        if flag is None:
            flag = _EMPTY_FLAG[key] = torch.empty(0, dtype=torch.int32, device=dev)
    (_fast_mod or _fast()).mc_calibration_update(preds, target, ws.cand, conf, acc, ws.notprob, ws.slot, flag)
    if not torch.cuda.is_current_stream_capturing():  # captured: the kernel side runs the one-word protocol
        ws.slot ^= 1
    return conf, acc


# ------------------------------------------------------------------------------------------------------ regression
# sum ids of csrc/regression/moments.hip
SSE, SAE, SP, ST, SPP, STT, SPT, MAPE, SMAPE, SABST, MSLE, LOGCOSH, MINK, COUNT = range(14)
# the centred sums' unshifted twins (a Pearson fold and raw-sum destinations sharing one pass)
SP0, ST0, SPP0, STT0, SPT0 = range(14, 19)
_UNSHIFTED = {SP: SP0, ST: ST0, SPP: SPP0, STT: STT0, SPT: SPT0}
FOLD_NONE, FOLD_PEARSON = 0, 1


def sum_diff(a: int, b: int) -> int:
    """Destination id meaning ``sum[a] - sum[b]`` (e.g. ``sum_diff(ST, SP)`` = Σ(t - p))."""
    return 32 + 32 * int(a) + int(b)


def _sum_ids(i: int) -> "tuple[int, ...]":
    return (i,) if i < 32 else ((i - 32) // 32, (i - 32) % 32)


def _unshifted_id(i: int) -> int:
    """The same destination id reading the unshifted twins of the centred sums."""
    if i < 32:
        return _UNSHIFTED.get(i, i)
    a, b = (i - 32) // 32, (i - 32) % 32
    return sum_diff(_UNSHIFTED.get(a, a), _UNSHIFTED.get(b, b))


def moments_update(
    preds: Tensor,
    target: Tensor,
    num_outputs: int,
    sums: "list[int]",
    dests: "list[Tensor]",
    dest_ids: "list[int]",
    eps: float = 1.17e-06,
    power: float = 2.0,
    shift_p: Optional[Tensor] = None,
    shift_t: Optional[Tensor] = None,
    want_sums: bool = False,
    fold: int = FOLD_NONE,
) -> Optional[Tensor]:
    """One pass computing the requested per-output sums and adding ``sum[dest_ids[j]]`` into ``dests[j]``.

    ``preds``/``target`` are ``[N, num_outputs]`` (or 1-D). Returns the ``[num_outputs, 19]`` fp64 sums if asked.
    ``dest_ids`` entries may be :func:`sum_diff` pairs.  ``fold=FOLD_PEARSON`` additionally folds the batch into the
    six running Pearson states given FIRST in ``dests`` (``[mean_x, mean_y, m2_x, m2_y, c_xy, n]``, in place;
    ``shift_p``/``shift_t`` must be the current means); ``dest_ids`` then names the remaining destinations.
    """
    mask = 0
    for s in list(sums) + [j for i in dest_ids for j in _sum_ids(int(i))]:
        mask |= 1 << int(s)
    if fold == FOLD_PEARSON:
        mask |= (1 << SP) | (1 << ST) | (1 << SPP) | (1 << STT) | (1 << SPT) | (1 << COUNT)
    needs_grad = torch.is_grad_enabled() and (preds.requires_grad or target.requires_grad)
    if preds.is_cuda and not needs_grad:
        if preds.dtype != target.dtype or not preds.is_floating_point():
            dt = torch.promote_types(preds.dtype, target.dtype)
            dt = dt if dt.is_floating_point else torch.float32
            preds, target = preds.to(dt), target.to(dt)
        res = (_fast_mod or _fast()).moments_update(
            preds, target, num_outputs, mask, float(eps), float(power), shift_p, shift_t,
            dests if isinstance(dests, (list, tuple)) else list(dests),
            dest_ids if isinstance(dest_ids, (list, tuple)) else list(dest_ids), want_sums, fold,
        )
        return res if want_sums else None
    return _cpu.moments_update(preds, target, num_outputs, mask, eps, power, shift_p, shift_t, dests, dest_ids,
                               want_sums, fold)


class MomentsPlan:
    """One metric's request to the moments kernel, deferrable so a ``MetricCollection`` can merge the requests of
    all its streaming regression members on the same inputs into ONE :func:`moments_update` (one pass over the data,
    one or two launches for the whole collection)."""

    __slots__ = ("preds", "target", "k", "dests", "ids", "eps", "power", "fold_states", "shift_p", "shift_t", "src",
                 "checked", "_mask")

    def __init__(self, preds: Tensor, target: Tensor, k: int, dests: "list[Tensor]", ids: "list[int]",
                 eps: float = 1.17e-06, power: float = 2.0, fold_states: Optional["list[Tensor]"] = None,
                 shift_p: Optional[Tensor] = None, shift_t: Optional[Tensor] = None,
                 src: Optional[tuple] = None, checked: bool = False) -> None:
        self.preds, self.target, self.k = preds, target, k
        self.dests, self.ids = dests, ids
        self.eps, self.power = eps, power
        self.fold_states, self.shift_p, self.shift_t = fold_states, shift_p, shift_t
        self.src = src if src is not None else (preds, target)  # the caller's input objects (merge key)
        self.checked = checked  # destinations already validated (see states_ready)
        self._mask = None

    def deferrable(self) -> bool:
        p, t = self.preds, self.target
        if not (p.is_cuda and t.is_cuda) or (torch.is_grad_enabled() and (p.requires_grad or t.requires_grad)):
            return False
        if self.checked:
            return True
        dev = p.get_device()
        return all(d.get_device() == dev and d.is_contiguous() for d in self.dests + (self.fold_states or []))

    def _uses(self) -> int:
        m = self._mask
        if m is None or m[0] != len(self.ids):  # (ids only grow, by merging)
            bits = 0
            for i in self.ids:
                for j in _sum_ids(int(i)):
                    bits |= 1 << j
            m = self._mask = (len(self.ids), bits)
        return m[1]

    def key(self) -> tuple:
        """Plans merge when they read the same input objects with the same column count (and the same eps /
        power where those enter the sums).  Object identity is exact here: every plan of one collection update
        keeps its inputs alive until the merged call has run."""
        m = self._uses()
        eps = self.eps if m & ((1 << MAPE) | (1 << SMAPE)) else None
        power = self.power if m & (1 << MINK) else None
        return (id(self.src[0]), id(self.src[1]), self.k, eps, power)

    def run(self) -> None:
        fold = self.fold_states is not None
        moments_update(self.preds, self.target, self.k, [], (self.fold_states or []) + self.dests, self.ids,
                       eps=self.eps, power=self.power, shift_p=self.shift_p, shift_t=self.shift_t,
                       fold=FOLD_PEARSON if fold else FOLD_NONE)


def states_ready(owner: dict, states: tuple, dev: int, dtypes: tuple = (torch.float32, torch.float64, torch.int64)) -> bool:
    """True if ``states`` are contiguous tensors on CUDA device ``dev`` with an accepted dtype.  The verdict is cached
    in ``owner`` against the state OBJECTS (held, compared with ``is``): a metric's states stay the same objects
    across in-place kernel updates, so the per-update check is a few identity tests instead of ~4 tensor queries per
    state (host time is what bounds these updates)."""
    c = owner.get("_states_ready")
    if c is not None and c[0] == dev and len(c[1]) == len(states):
        for a, b in zip(c[1], states):
            if a is not b:
                break
        else:
            return True
    ok = all(t.is_cuda and t.get_device() == dev and t.is_contiguous() and t.dtype in dtypes for t in states)
    owner["_states_ready"] = (dev, states) if ok else None
    return ok


def run_moments_plans(plans: "list[MomentsPlan]", merged_out: Optional[list] = None) -> int:
    """Execute deferred plans, merging those on identical inputs (at most one Pearson fold and 32 plain
    destinations per launch).  Returns the number of kernel calls issued; ``merged_out`` receives the merged plans
    (``utils/fused_moments.py`` records a one-call step for replay)."""
    groups: "dict[tuple, list[MomentsPlan]]" = {}
    for pl in plans:
        groups.setdefault(pl.key(), []).append(pl)
    calls = 0
    for members in groups.values():
        while members:
            merged = MomentsPlan(members[0].preds, members[0].target, members[0].k, [], [], members[0].eps,
                                 members[0].power, src=members[0].src, checked=True)
            rest = []
            plain_ids: "list[bool]" = []  # per merged id: it came from a plan without a fold
            for pl in members:
                # the Pearson fold shifts the centred sums by the running means; plain destinations on the same pass
                # read the unshifted twins (SP0 ...) of those sums instead, so everything on these inputs is ONE pass
                if (pl.fold_states is not None and merged.fold_states is not None) or \
                        len(merged.dests) + len(pl.dests) > 32:
                    rest.append(pl)
                    continue
                merged.dests += pl.dests
                merged.ids += pl.ids
                plain_ids += [pl.fold_states is None] * len(pl.ids)
                if pl.fold_states is not None:
                    merged.fold_states, merged.shift_p, merged.shift_t = pl.fold_states, pl.shift_p, pl.shift_t
                if pl._uses() & ((1 << MAPE) | (1 << SMAPE)):
                    merged.eps = pl.eps
                if pl._uses() & (1 << MINK):
                    merged.power = pl.power
            if merged.fold_states is not None:
                merged.ids = [_unshifted_id(int(i)) if plain else i for i, plain in zip(merged.ids, plain_ids)]
                merged._mask = None
            merged.run()
            calls += 1
            if merged_out is not None:
                merged_out.append(merged)
            members = rest
    return calls


# ----------------------------------------------------------------------------------------------------------- image
def feature_moments_update(features: Tensor, feat_sum: Tensor, feat_cov: Tensor) -> None:
    """``feat_sum += Σ_n x_n`` and ``feat_cov += XᵀX`` in fp64 (fp64-MFMA SYRK on ROCm, upper triangle only)."""
    if features.is_cuda:
        if features.dtype not in (torch.float32, torch.float16, torch.bfloat16, torch.float64):
            features = features.float()
        _ops().feature_moments_update(features.contiguous(), feat_sum, feat_cov)
    else:
        _cpu.feature_moments_update(features, feat_sum, feat_cov)


_EMPTY_F64: dict = {}


def dgemm(a: Union[Tensor, Sequence[Tensor]], b: Union[Tensor, Sequence[Tensor]], out: Union[Tensor, Sequence[Tensor]],
          alpha: Union[float, Sequence[float]] = 1.0, beta: Union[float, Sequence[float]] = 0.0,
          cin: Optional[Union[Tensor, Sequence[Optional[Tensor]]]] = None,
          diag: Union[float, Sequence[float]] = 0.0) -> None:
    """``out_i = alpha_i a_i @ b_i + beta_i cin_i + diag_i I`` in fp64 on the matrix cores (``csrc/image/dgemm.hip``);
    one or two problems of one shape per launch.  CPU: the same formula with torch ops."""
    def seq(x, n):
        return list(x) if isinstance(x, (list, tuple)) else [x] * n

    single = isinstance(a, Tensor)
    a_l = [a] if single else list(a)
    n = len(a_l)
    b_l, o_l = seq(b, n) if not single else [b], seq(out, n) if not single else [out]
    al, be, dg, ci = seq(alpha, n), seq(beta, n), seq(diag, n), seq(cin, n)
    if a_l[0].is_cuda:
        dev = a_l[0].device
        empty = _EMPTY_F64.get(dev)
        if empty is None:
            empty = _EMPTY_F64[dev] = torch.empty(0, dtype=torch.float64, device=dev)
        _ops().dgemm_nn(a_l, b_l, o_l, [c if c is not None else empty for c in ci], [float(x) for x in al],
                        [float(x) for x in be], [float(x) for x in dg])
        return
    for i in range(n):
        r = al[i] * (a_l[i] @ b_l[i])
        if ci[i] is not None:
            r = r + be[i] * ci[i]
        if dg[i]:
            r = r + dg[i] * torch.eye(r.shape[0], r.shape[1], dtype=r.dtype)
        o_l[i].copy_(r)


def dgemv4_blocks(d: int, device: Optional[torch.device] = None) -> int:
    """Rows of per-block partial norms ``dgemv4_resid`` writes (1 on CPU)."""
    if device is not None and device.type != "cuda":
        return 1
    return int(_ops().dgemv4_blocks(d))


def euclid_f64(x: Tensor, y: Optional[Tensor], zero_diagonal: bool, sqrt: bool = True) -> Tensor:
    """Pairwise euclidean distances with the reference's fp64 formula (``F/pairwise/euclidean.py:35-44``):
    ``sqrt(f32(|x_i|^2 + |y_j|^2 - 2 x_i.y_j))`` with fp64 norms and an fp64-MFMA GEMM whose epilogue writes the fp32
    distances directly (``csrc/image/dgemm.hip`` ``euclid_f64``; ``y`` read as rows, no transposed copy).  Squared
    distances that round below zero are clamped to 0 (the reference returns NaN for them).  Returns fp32 ``[N, M]``."""
    x64 = x.to(torch.float64).contiguous()
    y64 = x64 if y is None or y is x else y.to(torch.float64).contiguous()
    nx = (x64 * x64).sum(1)
    ny = nx if y64 is x64 else (y64 * y64).sum(1)
    if x.is_cuda:
        out = torch.empty(x64.shape[0], y64.shape[0], dtype=torch.float32, device=x.device)
        _ops().euclid_f64(x64, y64, nx, ny, bool(zero_diagonal), bool(sqrt), out)
        return out
    d2 = (nx[:, None] + ny[None, :] - 2 * (x64 @ y64.T)).float().clamp_(min=0)
    if zero_diagonal:
        d2.fill_diagonal_(0)
    return d2.sqrt_() if sqrt else d2


def dgemv4_resid(a: Tensor, w_in: Tensor, part_in: Tensor, normalize: bool, w_out: Tensor, part_out: Tensor) -> None:
    """One power-iteration step on 4 vectors: ``w_out = v - a v`` with ``v = w_in / ||w_in||`` (column norms from the
    previous step's per-block partials ``part_in``); writes this step's partial squared norms into ``part_out``."""
    if a.is_cuda:
        _ops().dgemv4_resid(a, w_in, part_in, normalize, w_out, part_out)
        return
    v = w_in / part_in.sum(0).sqrt().clamp(min=1e-300) if normalize else w_in
    w_out.copy_(v - a @ v)
    part_out.copy_((w_out * w_out).sum(0, keepdim=True))


# ------------------------------------------------------------------------------ fused compute() of a collection
class _TaskRecorder:
    """Records the one-block reductions of ``stat_reduce`` / ``confmat_reduce`` / ``curve_score`` /
    ``regression_compute`` as task descriptors; :meth:`flush` runs all of them in ONE launch
    (``csrc/common/compute_tasks.hip``).  Output tensors are allocated at record time, so the callers get their
    results as views of tensors the flush fills."""

    def __init__(self, poison: bool = False) -> None:
        self.rows: list = []
        self.keep: list = []
        self.meta: list = []  # per row: (pointer-slot tensors, outputs) -- utils/fused_compute.py builds plans from it
        self.lds = 0
        self.anchor: Optional[Tensor] = None
        self.poison = poison

    def add(self, kind: int, blocks: int, ints: Sequence[int], floats: Sequence[float], tensors: Sequence[Optional[Tensor]],
            outs: Sequence[Tensor], lds: int) -> None:
        row = [kind, blocks] + [int(v) for v in ints] + [0] * (6 - len(ints))
        fl = list(floats) + [0.0] * (2 - len(floats))
        row += [struct.unpack("<q", struct.pack("<d", float(v)))[0] for v in fl]
        ptrs = [t.data_ptr() if t is not None else 0 for t in tensors]
        row += ptrs + [0] * (8 - len(ptrs))
        self.rows.append(row)
        self.meta.append((list(tensors), list(outs)))
        self.keep.extend(t for t in tensors if t is not None)
        self.lds = max(self.lds, lds)
        if self.anchor is None:
            self.anchor = outs[0]
        if self.poison:
            for o in outs:
                o.fill_(float("nan") if o.is_floating_point() else -(2**30))

    def flush(self) -> int:
        """Launch the recorded tasks (``ceil(n / 32)`` launches); returns the number of tasks."""
        n = len(self.rows)
        for i in range(0, n, 32):
            desc = torch.tensor(self.rows[i : i + 32], dtype=torch.int64)
            _ops().compute_tasks(desc, self.anchor, self.lds)
        self.rows, self.keep, self.meta = [], [], []
        return n


_RECORDER: Optional[_TaskRecorder] = None


class fused_compute:  # noqa: N801 - context manager
    """``with ops.fused_compute() as rec: ...; rec.flush()`` -- record instead of launching the fused reductions."""

    def __init__(self, poison: bool = False) -> None:
        self.rec = _TaskRecorder(poison)

    def __enter__(self) -> _TaskRecorder:
        global _RECORDER
        self._prev = _RECORDER
        _RECORDER = self.rec
        return self.rec

    def __exit__(self, *exc) -> None:
        global _RECORDER
        _RECORDER = self._prev


_TASK_STAT, _TASK_CONFMAT, _TASK_CURVE, _TASK_REG_F32, _TASK_REG_F64 = 0, 1, 2, 3, 4
_TASK_RATIO_F32, _TASK_RATIO_F64, _TASK_STAT_SCORES = 5, 6, 7
_N_KIND = {torch.float32: 1, torch.float64: 2, torch.int64: 3}


def ratio(a: Tensor, b: Union[Tensor, int, float], take_sqrt: bool = False) -> Tensor:
    """``a / b`` (then ``sqrt``): the compute() of MSE / RMSE / MAE and similar running-sum metrics.  Eager ATen
    ops normally; inside :class:`fused_compute` a task of the one-launch compute kernel."""
    rec = _RECORDER
    if (rec is not None and isinstance(b, Tensor) and a.is_cuda and b.is_cuda and a.dtype in (torch.float32, torch.float64)
            and (b.dtype == torch.int64 or b.dtype == a.dtype) and a.is_contiguous() and b.is_contiguous()
            and 1 <= a.numel() <= (1 << 20) and (b.dim() == 0 or b.shape == a.shape)):
        out = torch.empty_like(a, memory_format=torch.contiguous_format)
        rec.add(_TASK_RATIO_F32 if a.dtype == torch.float32 else _TASK_RATIO_F64, 1,
                [a.numel(), _N_KIND[b.dtype], 1 if (b.dim() > 0 and b.numel() > 1) else 0, int(bool(take_sqrt))], [],
                [a, b, out], [out], 0)
        return out
    r = a / b
    return torch.sqrt(r) if take_sqrt else r


def stat_scores_output(tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, average: Optional[str]) -> Optional[Tensor]:
    """Recorded StatScores compute (global multidim, micro / macro / none) inside :class:`fused_compute`; None when
    not recording or not applicable (the caller then runs its ATen ops)."""
    rec = _RECORDER
    if rec is None or not tp.is_cuda or tp.dim() != 1 or average not in ("micro", "macro", "none", None):
        return None
    if not all(t.dtype == torch.int64 and t.is_contiguous() and t.shape == tp.shape for t in (tp, fp, tn, fn)):
        return None
    c = tp.numel()
    if c < 1:
        return None
    avg = {"micro": 0, "macro": 1}.get(average, 3)
    if avg == 3:
        out = torch.empty(c, 5, dtype=torch.int64, device=tp.device)
    else:
        out = torch.empty(5, dtype=torch.float32 if avg == 1 else torch.int64, device=tp.device)
    rec.add(_TASK_STAT_SCORES, 1, [c, avg], [], [tp, fp, tn, fn, out], [out], 0)
    return out


# --------------------------------------------------------------------------------------- confmat reductions
CM_JACCARD, CM_KAPPA, CM_MCC = 0, 1, 2
_CM_AVG = {"micro": 0, "macro": 1, "weighted": 2, "none": 3, None: 3}
_KAPPA_W = {None: 0, "none": 0, "linear": 1, "quadratic": 2}


def confmat_reducible(confmat: Tensor) -> bool:
    return confmat.is_cuda and confmat.dim() == 2 and confmat.dtype == torch.int64 and 2 <= confmat.shape[0] <= 4096 \
        and confmat.shape[0] == confmat.shape[1]


def confmat_reduce(confmat: Tensor, kind: int, average: Optional[str] = "macro", ignore_index: Optional[int] = None,
                   weights: Optional[str] = None) -> Tensor:
    """Jaccard / Cohen kappa / MCC of a ROCm ``[C, C]`` int64 confusion matrix in one launch
    (``csrc/classification/confmat_reduce.hip``).  Jaccard returns the per-class ``[C]`` vector for average none."""
    c = confmat.shape[0]
    out = torch.empty(c + 1, dtype=torch.float32, device=confmat.device)
    rec = _RECORDER
    if rec is not None and confmat.is_cuda and confmat_reducible(confmat):
        cm = confmat.contiguous()
        rec.add(_TASK_CONFMAT, 1, [c, kind, _CM_AVG[average], -1 if ignore_index is None else int(ignore_index),
                                   _KAPPA_W[weights]], [], [cm, out], [out], 3 * c * 8)
    else:
        (_fast_mod or _fast()).confmat_reduce(confmat.contiguous(), kind, _CM_AVG[average],
                                              -1 if ignore_index is None else int(ignore_index), _KAPPA_W[weights], out)
    if kind == CM_JACCARD:
        return out[:c] if average in (None, "none") else out[c]
    return out[0]


def calibration_bins(conf: Tensor, acc: Tensor, bounds: Tensor) -> Tensor:
    """``[len(bounds), 3]`` (count, Σconf, Σacc) per ``bucketize(conf, bounds, right=True) - 1`` bin, one pass."""
    nb = bounds.numel()
    sums = torch.zeros(nb, 3, dtype=torch.float32, device=conf.device)
    bad = torch.zeros(1, dtype=torch.int32, device=conf.device)
    (_fast_mod or _fast()).calibration_bins(conf.contiguous(), acc.contiguous(), bounds.float().contiguous(), sums,
                                            bad)
    return sums


# ------------------------------------------------------------------------------------- regression ratio scores
REG_EV, REG_R2, REG_PEARSON, REG_CONCORDANCE = 0, 1, 2, 3
MULTIOUT_IDS = {"raw_values": 0, "uniform_average": 1, "variance_weighted": 2}
_REG_STATE_DTYPES = (torch.float32, torch.float64)
_REG_N_DTYPES = (torch.float32, torch.float64, torch.int64)


def regression_computable(states: Sequence[Tensor], n: Union[Tensor, int, float]) -> bool:
    """True when :func:`regression_compute` takes these states: ROCm, contiguous, one f32/f64 dtype, equal sizes."""
    s0 = states[0]
    if not s0.is_cuda or s0.dtype not in _REG_STATE_DTYPES or not s0.is_contiguous():
        return False
    dev, k, dt = s0.get_device(), s0.numel(), s0.dtype
    if k < 1 or k > (1 << 20):
        return False
    for s in states[1:]:
        if not (s.is_cuda and s.get_device() == dev and s.dtype == dt and s.numel() == k and s.is_contiguous()):
            return False
    if isinstance(n, Tensor):
        return (n.is_cuda and n.get_device() == dev and n.dtype in _REG_N_DTYPES and n.numel() in (1, k)
                and n.is_contiguous())
    return isinstance(n, (int, float))


def regression_compute(kind: int, states: Sequence[Tensor], n: Union[Tensor, int, float], multioutput: int,
                       bound: float = 0.0) -> Tensor:
    """Explained variance / R^2 / Pearson / concordance from their running sums in one launch
    (``csrc/regression/regression_compute.hip``).  Returns ``[k + 2]``: the per-output scores, the
    ``multioutput`` average and the flag (Pearson / concordance: a variance below ``bound``; R^2: fewer than two
    samples)."""
    s0 = states[0]
    out = torch.empty(s0.numel() + 2, dtype=s0.dtype, device=s0.device)
    rec = _RECORDER
    if rec is not None and s0.is_cuda and regression_computable(states, n):
        k = s0.numel()
        need = {REG_EV: 4, REG_R2: 3}.get(kind, 5)
        st = list(states[:need]) + [states[0]] * (5 - need)
        if isinstance(n, Tensor):
            n_kind = {torch.float32: 1, torch.float64: 2, torch.int64: 3}[n.dtype]
            n_per_col = 1 if (n.numel() == k and k > 1) else 0
            n_t, n_val = n, 0.0
        else:
            n_kind, n_per_col, n_t, n_val = 0, 0, None, float(n)
        rec.add(_TASK_REG_F32 if s0.dtype == torch.float32 else _TASK_REG_F64, 1,
                [kind, k, n_kind, n_per_col, int(multioutput)], [n_val, bound], st + [n_t, out], [out], 0)
    elif isinstance(n, Tensor):
        (_fast_mod or _fast()).regression_compute(kind, states, n, 0.0, multioutput, bound, out)
    else:
        (_fast_mod or _fast()).regression_compute(kind, states, None, float(n), multioutput, bound, out)
    return out


_CALIB_WS: dict = {}


def calibration_error_l1_max(conf: Tensor, acc: Tensor, bounds: Tensor, norm: str) -> Tensor:
    """``l1`` / ``max`` calibration error of ROCm f32 confidences in two launches (bins + one-block reduce).

    The (count, Σconf, Σacc) bins live in a per-(n_bins, device, stream) workspace that the reduce kernel zeroes
    after reading it: no allocation or fill launch per compute()."""
    nb = bounds.numel()
    key = (nb, conf.device, torch.cuda.current_stream(conf.device).cuda_stream)
    ws = _CALIB_WS.get(key)
    if ws is None:
        ws = _CALIB_WS[key] = (torch.zeros(nb, 3, dtype=torch.float32, device=conf.device),
                               torch.zeros(1, dtype=torch.int32, device=conf.device))
    sums, bad = ws
    b = bounds if (bounds.dtype == torch.float32 and bounds.is_contiguous()) else bounds.float().contiguous()
    f = _fast_mod or _fast()
    f.calibration_bins(conf.contiguous(), acc.contiguous(), b, sums, bad)
    out = torch.empty(1, dtype=torch.float32, device=conf.device)
    f.calibration_reduce_clear(sums, 0 if norm == "l1" else 1, out)
    return out[0]


def calibration_error_from_bins(sums: Tensor, norm: str) -> Tensor:
    """``l1`` / ``max`` calibration error of ROCm f32 ``[nb, 3]`` (count, Σconf, Σacc) bins in one launch (the bins
    are left untouched: incremental caches keep accumulating into them)."""
    out = torch.empty(1, dtype=torch.float32, device=sums.device)
    (_fast_mod or _fast()).calibration_reduce(sums, 0 if norm == "l1" else 1, out)
    return out[0]


def calibration_bins_into(conf: Tensor, acc: Tensor, bounds: Tensor, sums: Tensor) -> None:
    """Add the (count, Σconf, Σacc) bins of ROCm f32 ``conf`` / ``acc`` into ``sums`` ``[nb, 3]`` (one launch)."""
    key = ("bad", conf.device)
    bad = _CALIB_WS.get(key)
    if bad is None:
        bad = _CALIB_WS[key] = torch.zeros(1, dtype=torch.int32, device=conf.device)
    (_fast_mod or _fast()).calibration_bins(conf, acc, bounds, sums, bad)


RANK_COVERAGE, RANK_LRAP, RANK_LOSS = 0, 1, 2
_RANK_MAX_LABELS = 2048


def label_ranking_rows(preds: Tensor, target: Tensor, mode: int) -> Optional["tuple[Tensor, Tensor]"]:
    """Per-row coverage / LRAP / ranking loss of ROCm ``[M, L]`` scores (``csrc/classification/ranking.hip``: one
    wave per row, all-pairs counting in LDS).  Returns ``(values f64 [M], valid u8 [M])`` or None when the kernel does
    not apply (CPU tensors, L > 2048, non-float scores)."""
    if not (preds.is_cuda and preds.dim() == 2 and preds.dtype in (torch.float32, torch.float16, torch.bfloat16,
                                                                     torch.float64)
            and 1 <= preds.shape[1] <= _RANK_MAX_LABELS and not target.is_floating_point()):
        return None
    m = preds.shape[0]
    out = torch.empty(m, dtype=torch.float64, device=preds.device)
    valid = torch.empty(m, dtype=torch.uint8, device=preds.device)
    p = preds.contiguous()
    gmin = p.min().reshape(1) if (mode == RANK_COVERAGE and m) else p.new_zeros(1)
    _ops().label_ranking(p, target.contiguous(), mode, gmin, out, valid)
    return out, valid


_TOPK_MAX = 16


def topk_labels(preds: Tensor, k: int) -> Optional[Tensor]:
    """Column indices of the ``k`` largest scores per row of ROCm ``[N, C]`` scores, descending, as int32 ``[N, k]``
    (``csrc/classification/topk.hip``: one wave per row, register top-k per lane + k wave arg-max rounds; NaN ranks
    highest, ties go to the smaller column).  None when the kernel does not apply (CPU, k > 16, f64 / int scores)."""
    if not (preds.is_cuda and preds.dim() == 2 and preds.dtype in (torch.float32, torch.float16, torch.bfloat16)
            and 1 <= k <= min(_TOPK_MAX, preds.shape[1])):
        return None
    return _ops().topk_labels(preds.contiguous(), int(k))


def mc_topk_update(preds: Tensor, target: Tensor, ws: Tensor, flag: Tensor, k: int, ignore_index: Optional[int],
                   samplewise: bool) -> bool:
    """top_k > 1 multiclass stats fused with the top-k selection (``csrc/classification/topk.hip``): accumulates the
    ``[G, 3C + 1]`` :func:`mc_update` stats workspace from ROCm ``[N, C]`` scores and ``[N]`` targets.  Returns False
    (nothing done) when the kernel does not apply; the caller then takes topk + :func:`mc_update`."""
    if not (preds.is_cuda and preds.dim() == 2 and target.dim() == 1
            and preds.dtype in (torch.float32, torch.float16, torch.bfloat16)
            and 2 <= k <= min(_TOPK_MAX, preds.shape[1]) and not target.is_floating_point()):
        return False
    _ops().mc_topk_update(preds.contiguous(), target.contiguous(), ws, flag, int(k),
                          0 if ignore_index is None else int(ignore_index), ignore_index is not None, samplewise)
    return True


# -------------------------------------------------------------------------------------------- curve scores
SCORE_AUROC, SCORE_AP = 0, 1
_AVG_IDS = {None: 0, "none": 0, "macro": 1, "weighted": 2}


def curve_score(state: Tensor, kind: int, average: Optional[str]) -> "tuple[Tensor, Tensor, Tensor]":
    """AUROC / AP of a binned ``[T, C, 2, 2]`` ROCm state in one launch (``csrc/classification/curve.hip``).

    Returns ``(per_class [C], reduced [] , nan_flag i32 [1])``; ``reduced`` is the nan-aware macro / weighted
    average (undefined for ``average`` none)."""
    c = state.shape[1]
    out = torch.empty(c + 1, dtype=torch.float32, device=state.device)
    flag = torch.empty(1, dtype=torch.int32, device=state.device)
    st = state if state.is_contiguous() else state.contiguous()
    rec = _RECORDER
    if (rec is not None and st.is_cuda and st.dtype == torch.int64 and st.dim() == 4 and st.shape[2:] == (2, 2)
            and st.shape[0] >= 1 and 1 <= c <= 16384):
        rec.add(_TASK_CURVE, 1, [st.shape[0], c, kind, _AVG_IDS[average]], [], [st, out, flag], [out, flag], 8 * c)
    else:
        (_fast_mod or _fast()).curve_score(st, kind, _AVG_IDS[average], out, flag)
    return out[:c], out[c], flag


# ------------------------------------------------------------------------------------------- classification curves
CURVE_BINARY = 0
CURVE_MULTILABEL = 1
CURVE_MULTICLASS = 2


def curve_update(preds: Tensor, target: Tensor, thr_sorted: Tensor, perm: Tensor, hist: Tensor, ctl: Tensor,
                 state: Tensor, err: Tensor, mode: int, ignore_index: Optional[int], micro: bool = False) -> None:
    """Binned multi-threshold confusion matrices ``state[T, H, 2, 2] += ...`` (``csrc/classification/curve.hip``).

    ``preds``: ``[N]`` (binary), ``[N, L]`` (multilabel) or ``[N, C]`` (multiclass) raw scores; sigmoid / softmax is
    applied on the device iff any considered score is outside ``[0, 1]``.  ``thr_sorted`` (f64, ascending) and
    ``perm`` (caller index of each sorted threshold) describe the thresholds.  ``hist`` / ``ctl`` are int32 scratch
    that must be zero on entry and are zero again on exit.  Invalid targets set bits in ``err``.
    """
    if preds.is_cuda:
        if preds.dtype not in (torch.float32, torch.float16, torch.bfloat16, torch.float64):
            preds = preds.float()
        if target.dtype == torch.bool:
            target = target.to(torch.uint8)
        _ops().curve_update(preds.contiguous(), target.contiguous(), thr_sorted, perm, hist, ctl, state, err,
                            mode, -1 if ignore_index is None else int(ignore_index), ignore_index is not None, micro)
    else:
        _cpu.curve_update(preds, target, thr_sorted, perm, state, err, mode, ignore_index, micro)


# ----------------------------------------------------------------------------------------------- image windows
SSIM_MODE = 0
UQI_MODE = 1
VIF_MODE = 2
SCC_MODE = 3


def ssim2d_partials(x: Tensor, y: Tensor, wh: Tensor, ww: Tensor, c12: Tensor, mode: int = SSIM_MODE) -> Tensor:
    """Per-plane sums of SSIM (or UQI) and contrast sensitivity over all windows fully inside the image.

    ``x``/``y``: ``[P, H, W]``; ``wh``/``ww``: separable window weights; ``c12``: ``(c1, c2, eps)`` as a tensor (may
    live on the device).  Returns ``[P, T, 2]`` partial sums (``T`` tiles on ROCm, 1 on the CPU); callers sum dim 1.
    """
    if x.is_cuda:
        acc = torch.float64 if x.dtype == torch.float64 else torch.float32
        if x.dtype not in (torch.float32, torch.float16, torch.bfloat16, torch.float64):
            x, y = x.float(), y.float()
        return _ops().ssim2d_partials(x.contiguous(), y.contiguous(), wh.to(acc).contiguous(),
                                      ww.to(acc).contiguous(), c12.to(device=x.device, dtype=acc).contiguous(), mode)
    return _cpu.ssim2d_partials(x, y, wh, ww, c12, mode)


# ------------------------------------------------------------------------------------------------------- detection
BOX_IOU, BOX_GIOU, BOX_DIOU, BOX_CIOU = range(4)


def box_pairwise(a: Tensor, b: Tensor, op: int = BOX_IOU, aligned: bool = False) -> Tensor:
    """IoU-family matrix ``[N, M]`` (or ``[N]`` for aligned pairs) of xyxy boxes (``csrc/detection/box_ops.hip``)."""
    if a.is_cuda:
        dt = a.dtype if a.dtype in (torch.float32, torch.float16, torch.bfloat16, torch.float64) else torch.float32
        return _ops().box_pairwise(a.to(dt).contiguous(), b.to(dt).contiguous(), op, aligned)
    return _cpu.box_pairwise(a, b, op, aligned)


def expected_mutual_info(a: Tensor, b: Tensor, n: float) -> Tensor:
    """Expected mutual information of clusterings with fp64 sizes ``a`` [R] / ``b`` [C] over ``n`` samples, one kernel
    (``csrc/clustering/emi.hip``); fp64 0-d on the device."""
    return _ops().expected_mutual_info(a, b, float(n))


def map_pack(preds: Any, target: Any, box_mode: int) -> Any:
    """MeanAveragePrecision.update's per-image validation + packing into the 7 flat bbox states in one native call
    (``csrc/bindings/fastcall.cpp`` map_pack): ``(7 flat tensors, det_sizes, gt_sizes)`` or None where the batch is
    not a regular ROCm batch (the caller's Python path handles it)."""
    mod = _fast_mod or _fast()
    fn = getattr(mod, "map_pack", None)
    return fn(preds, target, int(box_mode)) if fn is not None else None


def box_pairwise_ragged(a: Tensor, b: Tensor, a_off: Tensor, b_off: Tensor, o_off: Tensor, a_lab: Tensor,
                        b_lab: Tensor, op: int, threshold: Optional[float], invalid: float, total: int) -> Tensor:
    """IoU-family matrices of a ragged batch of images in one flat ``[sum n_i m_i]`` tensor (image i's ``[n_i, m_i]``
    matrix at ``o_off[i]``), values ``< threshold`` and label mismatches (when labels are given, i.e. non-empty) set to
    ``invalid`` (``csrc/detection/box_ops.hip``).  ``total`` = ``o_off[-1]`` (known on the host: no device read)."""
    if a.is_cuda:
        return _ops().box_pairwise_ragged(a.contiguous(), b.contiguous(), a_off, b_off, o_off, a_lab, b_lab, op,
                                          0.0 if threshold is None else float(threshold), threshold is not None,
                                          float(invalid), int(total))
    return _cpu.box_pairwise_ragged(a, b, a_off, b_off, o_off, a_lab, b_lab, op, threshold, invalid)


def iou_class_reduce(vals: Tensor, o_off: Tensor, b_off: Tensor, gt_lab: Tensor, classes: Tensor,
                     invalid: float) -> Tuple[Tensor, Tensor]:
    """fp64 sums and int64 counts of the valid (``!= invalid``) values of ragged IoU matrices: per class of the column's
    ground-truth label (slots ``[0, K)``, ``classes`` sorted) and overall (slot ``K``)."""
    if vals.is_cuda:
        return _ops().iou_class_reduce(vals, o_off, b_off, gt_lab, classes, float(invalid))
    return _cpu.iou_class_reduce(vals, o_off, b_off, gt_lab, classes, invalid)


def nms(boxes: Tensor, scores: Tensor, iou_threshold: float, idxs: Optional[Tensor] = None) -> Tensor:
    """Greedy NMS: indices of the kept ``[N, 4]`` xyxy boxes in descending score order (equal scores: lower index
    first).  With ``idxs`` only boxes of the same class suppress each other.  ROCm: bitmask-tile kernel + one-wave
    scan (``csrc/detection/nms.hip``); CPU: the same greedy rule in a native host loop (Python fallback: over the IoU
    matrix)."""
    if boxes.is_cuda or native_available():  # CPU: native host greedy loop (csrc/detection/nms_host.cpp)
        empty = boxes.new_empty(0, dtype=torch.long)
        return _ops().nms(boxes.contiguous(), scores.contiguous(), empty if idxs is None else idxs.contiguous(),
                          float(iou_threshold))
    return _cpu.nms(boxes, scores, iou_threshold, idxs)


def coco_match(dbox, darea, gbox, garea, gcrowd, det_start, det_cnt, gt_start, gt_cnt, area_rng, iou_thr,
               iou_pre=None, iou_off=None):
    """COCO greedy matching of every (image x class group, area range, IoU threshold); returns ``(dt_match, dt_ig)``
    uint8 ``[T, A, D]``.  Detections must be grouped and score-sorted, ground truths grouped in annotation order.

    ``iou_pre`` / ``iou_off`` optionally give precomputed per-group IoU blocks (``[det_cnt, gt_cnt]`` row-major at
    ``iou_off[group]``), e.g. mask IoUs for ``iou_type="segm"``; otherwise COCO box IoU is computed from ``dbox``.
    """
    if dbox.is_cuda or load_native(strict=False):
        # ROCm: one thread per (group, area, threshold); CPU: native host matcher (csrc/detection/coco_match_host.cpp)
        return _ops().coco_match(dbox, darea, gbox, garea, gcrowd, det_start, det_cnt, gt_start, gt_cnt, area_rng,
                                 iou_thr, iou_pre, iou_off)
    return _cpu.coco_match(dbox, darea, gbox, garea, gcrowd, det_start, det_cnt, gt_start, gt_cnt, area_rng, iou_thr,
                           iou_pre, iou_off)


def small_unique(a: Tensor, b: Tensor) -> Optional[Tuple[List[int], Tensor]]:
    """Sorted distinct values of two integer label tensors (ROCm, values in [0, 65536), at most 4096 of them) with ONE
    launch and one device->host copy (``csrc/detection/coco_prepare.hip`` small_unique_kernel): ``(host list, device
    int64 tensor)``; None where it does not apply (the caller takes ``torch.unique``)."""
    if not a.is_cuda or a.dtype.is_floating_point or b.dtype.is_floating_point or b.device != a.device:
        return None
    out = _ops().small_unique(a.reshape(-1).contiguous(), b.reshape(-1).contiguous())
    host = out.cpu()
    n = int(host[0])
    if n < 0:
        return None
    return host[1:1 + n].tolist(), out[1:1 + n]


def coco_prepare(classes: Tensor, off: Tensor, d_lab: Tensor, d_score: Tensor, d_box: Tensor, g_lab: Tensor,
                 g_box: Tensor, g_crowd: Tensor, g_area: Tensor, areas: Tensor, n_img: int, max_det: int,
                 max_per_image: int) -> List[Tensor]:
    """COCO grouping stage in one launch (``csrc/detection/coco_prepare.hip``): detections and ground truths in
    (image, category, score) matcher order with the group tables and the non-ignored ground-truth histogram.  Returns
    ``[tables int32 [4 G + A K], d_box, d_area, rank, cls, score, key2, g_box, g_area, g_crowd]`` (see the kernel)."""
    return _ops().coco_prepare(classes, off, d_lab, d_score, d_box, g_lab, g_box, g_crowd, g_area, areas, int(n_img),
                               int(max_det), int(max_per_image))


def coco_accumulate(dt_match: Tensor, dt_ig: Tensor, o: Tensor, rank_s: Tensor, score_s: Tensor, cls_s: Tensor,
                    npig: Tensor, r_thr: Tensor, max_dets: Sequence[int], precision: Tensor, recall: Tensor,
                    scores: Tensor) -> bool:
    """COCO accumulation of every (category, IoU threshold, area, max-dets) in one launch
    (``csrc/detection/coco_accumulate.hip``).  ``dt_match`` / ``dt_ig`` uint8 ``[T, A, D]`` from :func:`coco_match`,
    ``o`` the permutation to detections sorted by (category, score) (``cls_s`` / ``rank_s`` / ``score_s`` already in
    that order; category ``K`` = sentinel, skipped); fills ``precision`` / ``scores`` ``[T, R, K, A, M]`` and
    ``recall`` ``[T, K, A, M]`` in place.  Returns False (nothing written) where the kernel does not apply: CPU,
    T * A > 63 or more than 8 max-dets values."""
    T, A, n = dt_match.shape
    K = npig.shape[1]
    if not dt_match.is_cuda or T * A > 63 or len(max_dets) > 8 or n == 0:
        return False
    tpb, fpb = _ops().coco_pack_bits(dt_match.contiguous(), dt_ig.contiguous())  # (matcher order, coalesced)
    tpb, fpb = tpb[o], fpb[o]
    seg = torch.zeros(K + 1, dtype=torch.int64, device=dt_match.device)
    torch.cumsum(histogram(cls_s, K), 0, out=seg[1:])  # (sentinel category K, sorted last: skipped)
    _ops().coco_accumulate(tpb, fpb, rank_s.to(torch.int64).contiguous(), score_s.to(torch.float64).contiguous(), seg,
                           npig.contiguous(), r_thr.contiguous(), torch.tensor(list(max_dets), dtype=torch.int64),
                           int(T), precision, recall, scores)
    return True


def coco_accumulate_sorted(dt_match: Tensor, dt_ig: Tensor, o: Tensor, rank_v: Tensor, score_v: Tensor,
                           cls_v: Tensor, npig: Tensor, r_thr: Tensor, max_dets: Sequence[int], precision: Tensor,
                           recall: Tensor, scores: Tensor) -> bool:
    """:func:`coco_accumulate` from matcher-order ``rank_v`` / ``score_v`` / ``cls_v`` and the accumulation order ``o``:
    the bit packing, the gathers and the category segments in ONE launch (``coco_pack_sorted``), then the
    accumulation kernel.  False (nothing written) where the kernel does not apply."""
    T, A, n = dt_match.shape
    K = npig.shape[1]
    if not dt_match.is_cuda or T * A > 63 or len(max_dets) > 8 or n == 0:
        return False
    tpb, fpb, rank_s, score_s, seg = _ops().coco_pack_sorted(dt_match.contiguous(), dt_ig.contiguous(), o.contiguous(),
                                                             rank_v.contiguous(), score_v.contiguous(),
                                                             cls_v.contiguous(), int(K))
    _ops().coco_accumulate(tpb, fpb, rank_s, score_s, seg, npig.contiguous(), r_thr.contiguous(),
                           torch.tensor(list(max_dets), dtype=torch.int64), int(T), precision, recall, scores)
    return True


def coco_summary(prec: Tensor, rec: Tensor, cprec: Tensor, crec: Tensor, m_ap: int) -> Optional[Tensor]:
    """Every sum COCO's summary and per-class numbers need, in one launch (``csrc/detection/coco_accumulate.hip``
    coco_summary_kernel): an fp64 vector ``[psp, pcp]`` (``[T, ceil(K / 4), A*M]``: partial sums / counts of the defined
    precision entries per group of 4 categories), ``[sr, cr]`` (``[T, A*M]``: recall over K), then
    ``[mps, mpc, mrs, mrc]`` (``[T, K]``: per-category precision at (area 0, max-dets ``m_ap``; ``m_ap < 0``: zeros)
    and recall at (area 0, last max-dets)).  None where the kernel does not apply (CPU tensors, A * M > 32)."""
    T, R, K, A, M = prec.shape
    if not prec.is_cuda or A * M > 32:
        return None
    return _ops().coco_summary(prec.contiguous(), rec.contiguous(), cprec.contiguous(), crec.contiguous(), int(m_ap))


def panoptic_tables(pcode: Tensor, tcode: Tensor) -> List[Tensor]:
    """Per-image pixel areas of predicted segments, target segments and segment pairs from int32 ``[B, P]`` segment
    codes (``csrc/detection/panoptic.hip``: LDS hash tables, one block per image).  Returns pair keys (int64:
    ``pred << 32 | target``) and counts ``[B, 4096]``, pred / target keys and counts ``[B, 1024]`` (empty slots: key
    -1), and an overflow flag."""
    return list(_ops().panoptic_tables(pcode, tcode))


def rle_encode(masks: List[Tensor]) -> List[Tensor]:
    """Run-length encode every ``[n_i, H_i, W_i]`` mask tensor into one int32 pack per image
    (``[n, H, W, areas(n), offsets(n+1), change positions...]``, ``csrc/detection/rle.hip``): ROCm kernels (one host
    sync per call, to size the packs) or the native host loop; a torch fallback without the library."""
    if not masks:
        return []
    if masks[0].is_cuda or load_native(strict=False):
        return list(_ops().rle_encode(list(masks)))
    return _cpu.rle_encode(masks)


def rle_iou(dbuf: Tensor, ddesc: Tensor, gbuf: Tensor, gdesc: Tensor, pd: Tensor, pg: Tensor, gcrowd: Tensor) -> Tensor:
    """fp64 mask IoU of every (detection ``pd[p]``, ground truth ``pg[p]``) pair from their RLE descriptors
    (``[N, 5]``: position start, change count, area, H, W); crowd ground truths divide by the detection area,
    mismatched sizes give -1 (pycocotools ``rleIou``)."""
    if pd.is_cuda or load_native(strict=False):
        return _ops().rle_iou(dbuf, ddesc, gbuf, gdesc, pd, pg, gcrowd)
    return _cpu.rle_iou(dbuf, ddesc, gbuf, gdesc, pd, pg, gcrowd)


# ------------------------------------------------------------------------------------------ distance transforms
_DT_METRICS = {"euclidean": 0, "taxicab": 1, "chessboard": 2}


def line_distance_transform(cost: Tensor, spacing: float, metric: str) -> Optional[Tensor]:
    """Exact 1-D transform along the last dim: ``out[..., j] = min_k combine(|j - k| * spacing, cost[..., k])``
    (squared-euclidean lower envelope / taxicab scans / chessboard min-max; ``csrc/segmentation/
    distance_transform.hip``, ROCm kernel or native host loop).  None when the native library is unavailable."""
    if cost.dtype not in (torch.float32, torch.float64) or not (cost.is_cuda or native_available()):
        return None
    n = cost.shape[-1]
    out = _ops().line_distance_transform(cost.reshape(-1, n).contiguous(), float(spacing), _DT_METRICS[metric])
    return out.reshape(cost.shape)


# -------------------------------------------------------------------------------------------------------- pairwise
# metric ids of csrc/pairwise/pairwise.hip
PW_L1, PW_L2, PW_LP, PW_LP_INT = range(4)
_PW_TILE = 64


def pairwise_distance(x: Tensor, y: Tensor, metric: int, p: float = 2.0, zero_diagonal: bool = False,
                      reduction: Optional[str] = None) -> Tensor:
    """``[N, M]`` L1 / L2 / Lp distance matrix (or its row ``sum`` / ``mean`` ``[N]``) in the input's dtype; the
    HIP kernel fuses root, ``zero_diagonal`` and the row reduction (``csrc/pairwise/pairwise.hip``)."""
    if not x.is_cuda:
        return _cpu.pairwise_distance(x, y, metric, p, zero_diagonal, reduction)
    if x.dtype not in (torch.float32, torch.float16, torch.bfloat16, torch.float64):
        x, y = x.float(), y.float()
    x, y = x.contiguous(), y.to(x.dtype).contiguous()
    acc = torch.float64 if x.dtype == torch.float64 else torch.float32
    if metric == PW_LP and float(p).is_integer() and 3 <= p <= 15:
        metric = PW_LP_INT
    n, m = x.shape[0], y.shape[0]
    reduce = reduction in ("sum", "mean")
    out = torch.empty(n, -(-m // _PW_TILE) if reduce else m, dtype=acc, device=x.device)
    _ops().pairwise_distance(x, y, out, int(metric), float(p), bool(zero_diagonal), reduce)
    if reduce:
        out = out.sum(1)
        if reduction == "mean":
            out = out / m
    return out.to(x.dtype)


def corr_merge(stacked: Tensor) -> Tensor:
    """Merge ``[6, W, k]`` stacked per-rank Pearson states (mean_x, mean_y, var_x, var_y, corr_xy, n) into ``[6, k]``
    in one launch (``csrc/regression/regression_compute.hip`` ``corr_merge``; CPU tensors: the same fold on the
    host)."""
    return _ops().corr_merge(stacked.contiguous())


# ------------------------------------------------------------------------------------------- MFMA GEMM epilogues
GEMM_STORE, GEMM_EUCLID, GEMM_COSINE, GEMM_POLY_SUM, GEMM_ROW_MIN, GEMM_ROW_SUM, GEMM_ROW_COL_MAX = range(7)


def row_norms(x: Tensor, inverse: bool = False, y: Optional[Tensor] = None) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    """fp32 squared row norms (or inverse norms ``1 / ||x_i||``) of a ``[..., D]`` operand, accumulated in fp32 from
    the operand's own dtype: one wave per row on ROCm (``csrc/pairwise/gemm_nt.hip`` ``row_norms``).  With ``y`` (same
    dtype and D): both operands' norms from ONE launch, returned as a pair."""
    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16, torch.float16) and (
            y is None or (y.dtype == x.dtype and y.is_cuda)):
        res = _ops().row_norms(x.contiguous(), None if y is None else y.contiguous(), 1 if inverse else 0)
        return res[0] if y is None else (res[0], res[1])

    def one(t: Tensor) -> Tensor:
        s = torch.linalg.vector_norm(t, 2, dim=-1, dtype=torch.float32).reshape(-1)
        return 1.0 / s if inverse else s * s

    return one(x) if y is None else (one(x), one(y))


def gemm_nt(x: Tensor, y: Tensor, kind: int, aux_x: Optional[Tensor] = None, aux_y: Optional[Tensor] = None,
            scale: float = 1.0, coef: float = 0.0, degree: int = 1, zero_diagonal: bool = False,
            sqrt_out: bool = True, idx_x: Optional[Tensor] = None, idx_y: Optional[Tensor] = None,
            out_dtype: Optional[torch.dtype] = None) -> Tensor:
    """``X @ Y^T`` (``[N, D] x [M, D]`` or batched ``[B, N, D] x [B, M, D]``) with a fused epilogue
    (``csrc/pairwise/gemm_nt.hip``).  fp32 operands run v_mfma_f32_32x32x2f32; bf16 / fp16 operands run the 16-bit
    matrix cores (v_mfma_f32_32x32x16_{bf16,f16}, fp32 accumulate) straight from the 16-bit tensors -- no upcast copy.

    ``kind``: ``GEMM_STORE`` (scale * dot), ``GEMM_EUCLID`` (aux = squared row norms; sqrt(|x|^2 + |y|^2 - 2 x.y),
    exact recompute under cancellation), ``GEMM_COSINE`` (aux = inverse norms), ``GEMM_POLY_SUM`` (fp64 partial sums of
    ``(scale * dot + coef) ** degree`` per block, diagonal skipped with ``zero_diagonal``), ``GEMM_ROW_MIN``
    (``min_j 1 - |cos|`` partials ``[.., N, tiles]``), ``GEMM_ROW_SUM`` (row-sum partials of ``scale * dot``).
    ``idx_x`` / ``idx_y`` (int32 ``[B, rows]``): batch ``b`` multiplies the gathered rows ``x[idx_x[b]]`` and
    ``y[idx_y[b]]`` without materialising them (the caller guarantees the indices are in range).
    ``out_dtype``: the STORE / EUCLID / COSINE matrix's dtype: fp32 (default) or the operands' 16-bit dtype, rounded
    in the epilogue (no separate cast pass).
    """
    if x.is_cuda:
        # 16-bit operands of any width and alignment stay 16-bit (rows that are not 16-byte aligned are staged with
        # narrower DMA lanes in the kernel, csrc/pairwise/gemm_nt.hip GRAN): only mixed / other dtypes go to fp32
        h16 = x.dtype in (torch.bfloat16, torch.float16) and y.dtype == x.dtype and x.shape[-1] > 0
        if h16:
            x, y = x.contiguous(), y.contiguous()
        if not h16:
            x = x.float().contiguous()
            y = y.float().contiguous()
        out16 = 1 if (h16 and out_dtype == x.dtype and kind in (GEMM_STORE, GEMM_EUCLID, GEMM_COSINE)) else 0
        ax = None if aux_x is None else aux_x.float().contiguous()
        ay = None if aux_y is None else aux_y.float().contiguous()
        ix = None if idx_x is None else idx_x.to(torch.int32).contiguous()
        iy = None if idx_y is None else idx_y.to(torch.int32).contiguous()
        out = _ops().gemm_nt(x, y, int(kind), ax, ay, float(scale), float(coef), int(degree), bool(zero_diagonal),
                             bool(sqrt_out), ix, iy, out16)
        return out if out_dtype is None or out.dtype == out_dtype else out.to(out_dtype)
    if idx_x is not None:
        x, y = x[idx_x.long()], y[idx_y.long()]
    out = _cpu.gemm_nt(x, y, kind, aux_x, aux_y, scale, coef, degree, zero_diagonal, sqrt_out)
    return out if out_dtype is None or kind not in (GEMM_STORE, GEMM_EUCLID, GEMM_COSINE) else out.to(out_dtype)


def bert_rowcol_max(x: Tensor, y: Tensor) -> "tuple[Tensor, Tensor]":
    """Row / column maxima of ``x[b] @ y[b]^T`` for token sets of at most 128 per side (``csrc/text/bert_match.hip``,
    one block per pair, 64 x 64 MFMA super-tiles).  x ``[B, P, D]``, y ``[B, R, D]`` fp32, or bf16 / fp16 on the
    16-bit matrix cores (fp32 accumulate, maxima rounded to the input dtype); fp32 ``[B, P]`` / ``[B, R]`` out."""
    b, p, _ = x.shape
    r = y.shape[1]
    rmax = torch.empty(b, p, dtype=torch.float32, device=x.device)
    cmax = torch.empty(b, r, dtype=torch.float32, device=x.device)
    _ops().bert_rowcol_max(x.contiguous(), y.contiguous(), rmax, cmax)
    return rmax, cmax


def gemm_row_col_max(x: Tensor, y: Tensor, scale: float = 1.0) -> "tuple[Tensor, Tensor]":
    """``max_j scale * x_i.y_j`` per row and ``max_i`` per column of batched ``[B, N, D] x [B, M, D]`` fp32 operands
    from one MFMA GEMM launch whose epilogue keeps only the per-tile maxima (the ``[B, N, M]`` score matrix is never
    written), plus two tiny max reductions.  Returns ``(rows [B, N], cols [B, M])``."""
    b, n, m = x.shape[0], x.shape[1], y.shape[1]
    flat = gemm_nt(x, y, GEMM_ROW_COL_MAX, scale=scale)
    # partial counts follow the kernel's tile (128, or 256 for the large-problem kernel): the one that fits the output
    tm, tn = next((-(-m // t), -(-n // t)) for t in (128, 256)
                  if b * (n * -(-m // t) + -(-n // t) * m) == flat.numel())
    rows = flat[: b * n * tm].reshape(b, n, tm).amax(-1)
    cols = flat[b * n * tm:].reshape(b, tn, m).amax(1)
    return rows, cols


# ------------------------------------------------------------------------------------------------------------ text
_LEV_WAVES = 4  # waves (pairs) per block of csrc/text/levenshtein.hip (kWavesPerBlock)


def levenshtein(pred: Tensor, poff: Tensor, ref: Tensor, roff: Tensor, ins: int = 1, dele: int = 1, sub: int = 1,
                use_beam: bool = False, max_ref_len: Optional[int] = None) -> Tensor:
    """Batched edit distances ``[B]`` (int64) of int32 token-id sequences packed with int64 offsets
    (``csrc/text/levenshtein.hip``).  ROCm tensors run the wave-per-pair LDS kernel; CPU tensors run the native
    multithreaded host DP when the library is loaded, else the Python DP of :mod:`ops._cpu`."""
    out = torch.empty(poff.numel() - 1, dtype=torch.int64, device=pred.device)
    if max_ref_len is None:
        # the LDS rows are sized by the longest reference: the packed length bounds it with no device read (the
        # in-package callers pass the tokeniser's host-side maximum); only a bound too large for LDS reads the offsets
        bound = ref.numel()
        if roff.numel() <= 1:
            max_ref_len = 0
        elif not roff.is_cuda:
            max_ref_len = int((roff[1:] - roff[:-1]).max())
        elif _LEV_WAVES * 2 * (bound + 1) * 4 <= 160 * 1024:
            max_ref_len = bound
        else:
            max_ref_len = int((roff[1:] - roff[:-1]).max().item())
    args = (pred.int().contiguous(), poff.long().contiguous(), ref.int().contiguous(), roff.long().contiguous(), out,
            int(ins), int(dele), int(sub), bool(use_beam), int(max_ref_len))
    if pred.is_cuda or native_available():
        _ops().levenshtein(*args)
        return out
    _cpu.levenshtein(*args)
    return out


def eed_scores(hyps, refs, alpha: float, rho: float, deletion: float, insertion: float):
    """Extended edit distance of each (hypothesis, reference) string pair (native host DP, ``csrc/text/eed_host.cpp``)."""
    import numpy as np

    def pack(strs):
        arrs = [np.frombuffer(s.encode("utf-32-le"), dtype=np.uint32).astype(np.int32) for s in strs]
        off = np.zeros(len(arrs) + 1, dtype=np.int64)
        np.cumsum([len(a) for a in arrs], out=off[1:])
        ids = np.concatenate(arrs) if off[-1] else np.zeros(0, dtype=np.int32)
        return torch.from_numpy(ids), torch.from_numpy(off)

    h, ho = pack(hyps)
    r, ro = pack(refs)
    return _ops().eed_scores(h, ho, r, ro, float(alpha), float(rho), float(deletion), float(insertion)).tolist()


class _TokenNLL(torch.autograd.Function):
    """Autograd wrapper: forward = fused kernel (nll + per-row logsumexp), backward = (softmax - onehot) * g."""

    @staticmethod
    def forward(ctx, logits, target, ignore_index, flag):  # noqa: D102
        acc = torch.float64 if logits.dtype == torch.float64 else torch.float32
        nll = torch.empty(logits.shape[0], dtype=torch.float32, device=logits.device)
        lse = torch.empty(logits.shape[0], dtype=acc, device=logits.device)
        _ops().token_nll(logits, target, nll, lse, flag, 0 if ignore_index is None else int(ignore_index),
                         ignore_index is not None)
        ctx.save_for_backward(logits, target, lse)
        ctx.ignore_index = ignore_index
        return nll

    @staticmethod
    def backward(ctx, g):  # noqa: D102
        logits, target, lse = ctx.saved_tensors
        keep = torch.ones_like(target, dtype=torch.bool) if ctx.ignore_index is None else target != ctx.ignore_index
        gs = (g.to(lse.dtype) * keep)[:, None]
        grad = torch.exp(logits.to(lse.dtype) - lse[:, None]) * gs
        grad.scatter_add_(1, torch.where(keep, target, torch.zeros_like(target))[:, None], -gs)
        return grad.to(logits.dtype), None, None, None


def token_nll(logits: Tensor, target: Tensor, ignore_index: Optional[int], flag: Optional[Tensor] = None) -> Tensor:
    """Per-row ``-log softmax(logits)[target]`` (``[rows]`` fp32, 0 for ignored rows) -- fused single-pass HIP
    kernel on ROCm (``csrc/text/perplexity.hip``, differentiable via :class:`_TokenNLL`), fp32 ``log_softmax`` +
    gather on the host."""
    if logits.is_cuda:
        if flag is None:
            flag = torch.zeros(1, dtype=torch.int32, device=logits.device)
        return _TokenNLL.apply(logits.contiguous(), target.long().contiguous(), ignore_index, flag)
    return _cpu.token_nll(logits, target, ignore_index)


# ----------------------------------------------------------------------------------------------------------- audio
def _toeplitz_solve_kernel(r: Tensor, b: Tensor) -> Tensor:
    shape = r.shape
    rr = r.reshape(-1, shape[-1]).double().contiguous()
    bb = b.reshape(-1, shape[-1]).double().contiguous()
    x = torch.empty_like(rr)
    _ops().toeplitz_solve(rr, bb, x)
    return x.reshape(shape)


class _ToeplitzSolve(torch.autograd.Function):
    """x = T(r)^-1 b.  Backward: y = T^-1 g (T is symmetric), grad_b = y, grad_r[k] = -sum_{|i-j|=k} y_i x_j."""

    @staticmethod
    def forward(ctx, r, b):  # noqa: D102
        x = _toeplitz_solve_kernel(r, b)
        ctx.save_for_backward(r, x)
        return x

    @staticmethod
    def backward(ctx, g):  # noqa: D102
        r, x = ctx.saved_tensors
        y = _toeplitz_solve_kernel(r, g.contiguous())
        n = x.shape[-1]
        nfft = 1 << (2 * n - 1).bit_length()
        xf, yf = torch.fft.rfft(x, n=nfft), torch.fft.rfft(y, n=nfft)
        c_xy = torch.fft.irfft(xf * yf.conj(), n=nfft)[..., :n]  # sum_i y_i x_{i+k}
        c_yx = torch.fft.irfft(yf * xf.conj(), n=nfft)[..., :n]  # sum_i x_i y_{i+k}
        grad_r = -(c_xy + c_yx)
        grad_r[..., 0] = grad_r[..., 0] / 2
        return grad_r.to(r.dtype), y.to(r.dtype)


def toeplitz_solve(r: Tensor, b: Tensor) -> Tensor:
    """Solve ``T(r) x = b`` for batches of symmetric Toeplitz systems ``r, b: [..., L]`` (fp64): Levinson recursion,
    one wave per system on ROCm (``csrc/audio/levinson.hip``, differentiable); dense LU of the explicit matrix on the
    host."""
    if r.is_cuda:
        return _ToeplitzSolve.apply(r, b)
    return _cpu.toeplitz_solve(r, b)


def lpips_layer(f0: Tensor, f1: Tensor, w: Tensor, eps: float = 1e-8) -> Tensor:
    """``[N]`` spatial mean of ``sum_c w_c (f0/|f0| - f1/|f1|)^2`` for one LPIPS layer ``[N, C, H, W]`` -- fused
    single-pass HIP kernel on ROCm (``csrc/image/lpips.hip``), composite ATen ops on the host."""
    n, c = f0.shape[:2]
    pixels = f0[0, 0].numel()
    if f0.is_cuda:
        a = f0.reshape(n, c, pixels).contiguous()
        b = f1.to(a.dtype).reshape(n, c, pixels).contiguous()
        part = torch.empty(n, -(-pixels // 256), dtype=torch.float64, device=f0.device)
        _ops().lpips_layer(a, b, w.reshape(-1).float().contiguous(), part, float(eps))
        return (part.sum(1) / pixels).to(f0.dtype if f0.is_floating_point() else torch.float32)
    return _cpu.lpips_layer(f0, f1, w, eps)


def interp_mean(x: Tensor, xp: Tensor, fp: Tensor, offsets: Tensor) -> Tensor:
    """Mean over C ragged curves ``(xp, fp)[offsets[c]:offsets[c+1]]`` of their piecewise-linear interpolation at the
    grid ``x`` (``csrc/classification/curve_interp.hip``: one launch on ROCm, the same walk on the host)."""
    load_native(strict=True)
    return torch.ops.tm_amd.interp_mean(x.contiguous(), xp.contiguous(), fp.contiguous(), offsets.contiguous())


def stat_reduce(tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, kind: int, average: int, multilabel: bool,
                beta: float = 1.0) -> Tensor:
    """Fused stat-score compute on ``[R, C]`` int64 states (``csrc/classification/stat_reduce.hip``): ``[R]`` for
    micro / macro / weighted (ids 0 / 1 / 2), ``[R, C]`` for none (3)."""
    out = torch.empty(tp.shape[0] * (tp.shape[1] if average == 3 else 1), dtype=torch.float32, device=tp.device)
    rec = _RECORDER
    if (rec is not None and tp.is_cuda and tp.dim() == 2 and tp.shape[0] >= 1
            and all(t.dtype == torch.int64 and t.is_contiguous() and t.shape == tp.shape for t in (tp, fp, tn, fn))
            and 0 <= kind <= 5 and 0 <= average <= 3):
        rec.add(_TASK_STAT, tp.shape[0], [tp.shape[1], kind, average, int(bool(multilabel))], [float(beta) ** 2],
                [tp, fp, tn, fn, out], [out], 0)
    else:
        (_fast_mod or _fast()).stat_reduce(tp, fp, tn, fn, out, kind, average, multilabel, float(beta))
    return out.reshape(tp.shape[0], -1) if average == 3 else out


def biquad_cascade(x: Tensor, coefs: Tensor, rep: int, clamp: bool) -> Tensor:
    """Filter signals ``x [S, T]`` through per-filter cascades of biquads ``coefs [F, sections, 6]``
    ((b0, b1, b2, a0, a1, a2) per section); output row ``r`` = signal ``r // rep`` through filter ``r % F``
    (``csrc/audio/iir.hip``, fp64).  ``clamp`` clamps every section's output to [-1, 1] like
    ``torchaudio.functional.lfilter(clamp=True)``."""
    xs = x.double().contiguous()
    cf = coefs.double().contiguous()
    if xs.is_cuda:
        y = torch.empty(xs.shape[0] * rep, xs.shape[1], dtype=torch.float64, device=xs.device)
        _ops().biquad_cascade(xs, cf.to(xs.device), y, int(rep), bool(clamp))
        return y
    return _cpu.biquad_cascade(xs, cf, rep, clamp)


# ------------------------------------------------------------------------------------------------ audio / image
def snr_rows(preds: Tensor, target: Tensor, seg: int, scale_invariant: bool, zero_mean: bool, eps: float) -> Tensor:
    """SNR (``scale_invariant=False``) or SI-SDR-style ratio in dB per row of contiguous ``[rows, L]`` ROCm signals,
    one block per row (``csrc/audio/snr.hip``); ``seg``: zero-mean segment length (SA-SDR: per speaker)."""
    out = torch.empty(preds.shape[0], dtype=preds.dtype, device=preds.device)
    _ops().snr_rows(preds.contiguous(), target.contiguous(), out, int(seg), bool(scale_invariant), bool(zero_mean),
                    float(eps))
    return out


def inception_score(logits: Tensor, perm: Tensor, splits: int) -> Tensor:
    """(mean, std) Inception Score of ROCm ``[N, C]`` logits taken in ``perm`` order, ``torch.chunk`` splits
    (``csrc/image/inception_score.hip``, three launches)."""
    out = torch.empty(2, dtype=torch.float32, device=logits.device)
    _ops().inception_score(logits.contiguous(), perm.to(logits.device, torch.int64).contiguous(), int(splits), out)
    return out


def group_stats_update(preds: Tensor, target: Tensor, groups: Tensor, num_groups: int, threshold: float,
                       ignore_index: Optional[int], owner: dict, tp: Tensor, fp: Tensor, tn: Tensor,
                       fn: Tensor) -> None:
    """Per-group tp / fp / tn / fn of binary ROCm inputs added into the int64 ``[num_groups]`` states in place
    (``csrc/classification/group_stats.hip``: both score readings in one pass, LDS histogram, fold)."""
    ws = owner.get("_group_ws")
    if ws is None or ws[0].numel() != 8 * num_groups or ws[0].device != preds.device:
        ws = owner["_group_ws"] = (torch.zeros(8 * num_groups, dtype=torch.int64, device=preds.device),
                                   torch.zeros(1, dtype=torch.int32, device=preds.device))
    (_fast_mod or _fast()).group_stats_update(
        preds.reshape(-1).contiguous(), target.reshape(-1).contiguous(), groups.reshape(-1).to(torch.int64).contiguous(),
        int(num_groups), float(threshold), 0 if ignore_index is None else int(ignore_index), ignore_index is not None,
        ws[0], ws[1], tp, fp, tn, fn)


EM_MULTICLASS, EM_MULTILABEL, EM_LABELS = 0, 1, 2


def exact_match_update(preds: Tensor, target: Tensor, kind: int, C: int, P: int, threshold: float,
                       ignore_index: Optional[int], samplewise: bool, owner: dict,
                       correct: Optional[Tensor] = None, total: Optional[Tensor] = None) -> Optional[Tensor]:
    """Exact-match update of contiguous ROCm inputs (``csrc/classification/exact_match.hip``).  ``kind``
    EM_MULTICLASS: preds ``[N, C, P]`` scores, target ``[N, P]``; EM_MULTILABEL: preds / target ``[N, C, P]``;
    EM_LABELS: multiclass labels of any dtype, preds / target ``[N, C]`` (``C`` = positions, ``P`` = 1).  Global: ``correct`` / ``total`` int64 ``[1]`` states
    are updated in place, returns None.  Samplewise: returns the int64 ``[N]`` per-sample counts."""
    n = target.numel() // (P if kind == EM_MULTICLASS else C * P) if P and C else 0
    ws = owner.get("_em_ws")
    need = max(2, 2 * n)
    if ws is None or ws[0].numel() < need or ws[0].device != preds.device:
        ws = owner["_em_ws"] = (torch.zeros(need, dtype=torch.int64, device=preds.device),
                                torch.zeros(1, dtype=torch.int32, device=preds.device))
    out = torch.empty(n if samplewise else 0, dtype=torch.int64, device=preds.device)
    if correct is None:
        correct = total = ws[0][:1]  # unused by the samplewise fold
    (_fast_mod or _fast()).exact_match_update(
        preds, target, int(kind), int(C), int(P), kind == EM_MULTICLASS, float(threshold),
        0 if ignore_index is None else int(ignore_index), ignore_index is not None, bool(samplewise), ws[0], ws[1],
        correct, total, out)
    return out if samplewise else None


AGG_SUM, AGG_MEAN, AGG_MAX, AGG_MIN = 0, 1, 2, 3
AGG_NAN_ERROR, AGG_NAN_IGNORE, AGG_NAN_IMPUTE, AGG_NAN_WARN = 0, 1, 2, 3


def agg_update(x: Tensor, weight: Union[Tensor, float, None], kind: int, nan_mode: int, impute: float, owner: dict,
               s0: Tensor, s1: Optional[Tensor], flag: Tensor) -> Tensor:
    """One-launch aggregator update (``csrc/common/aggregate.hip``): NaN strategy, sum(x*w) / sum(w) / max / min
    in fp64 and the in-place state fold.  ``weight``: a python number (kernel argument), or a ROCm tensor of 1 or
    ``x.numel()`` elements.  Returns the int32 ``[2]`` control word whose element 1 holds this call's NaN count."""
    ws = owner.get("_agg_ws")
    if ws is None or ws[0].device != x.device:
        ws = owner["_agg_ws"] = (torch.empty(5 * 2048, dtype=torch.float64, device=x.device),
                                 torch.zeros(2, dtype=torch.int32, device=x.device))
    if isinstance(weight, Tensor):
        w, wconst = weight.reshape(-1).contiguous(), 1.0
    else:
        w = _EMPTY_F32.get(x.device)
        if w is None:
            w = _empty_f32(x.device)
        wconst = 1.0 if weight is None else float(weight)
    (_fast_mod or _fast()).agg_update(x.reshape(-1).contiguous(), w, wconst, int(kind), int(nan_mode), float(impute),
                                      ws[0], ws[1], s0, s0 if s1 is None else s1, flag)
    return ws[1]


_EMPTY_F32: dict = {}


def _empty_f32(device: torch.device) -> Tensor:
    t = _EMPTY_F32[device] = torch.empty(0, dtype=torch.float32, device=device)
    return t


HINGE_BINARY, HINGE_CRAMMER_SINGER, HINGE_ONE_VS_ALL = 0, 1, 2


def hinge_update(preds: Tensor, target: Tensor, mode: int, squared: bool, ignore_index: Optional[int], owner: dict,
                 measures: Tensor, total: Tensor, flag: Tensor) -> None:
    """Fused hinge-loss update of ROCm scores into the ``measures`` / ``total`` states (``csrc/classification/
    hinge.hip``): both readings of the scores (as given / sigmoid-or-softmax) accumulated in one pass, the fold keeps
    the one the batch calls for.  ``owner``: the metric's ``__dict__`` (holds the reusable workspace)."""
    k = measures.numel()
    ws = owner.get("_hinge_ws")
    if ws is None or ws[0].numel() != 2 * k + 1 or ws[0].device != preds.device:
        ws = owner["_hinge_ws"] = (torch.zeros(2 * k + 1, dtype=torch.float64, device=preds.device),
                                   torch.zeros(1, dtype=torch.int32, device=preds.device))
    _ops().hinge_update(preds, target, mode, bool(squared), 0 if ignore_index is None else int(ignore_index),
                        ignore_index is not None, ws[0], ws[1], measures, total, flag)


def stoi_segments(x_tob: Tensor, y_tob: Tensor, nframes: Tensor, extended: bool) -> Tensor:
    """Sum over each signal's valid 30-frame segments of the (extended) STOI segment correlation of ``[B, 15, F]``
    band envelopes (``csrc/audio/stoi.hip``); fp64 ``[B]``."""
    return _ops().stoi_segments(x_tob.contiguous(), y_tob.contiguous(), nframes.to(torch.int64).contiguous(),
                                bool(extended))


def linear_sum_assignment(cost: Tensor, maximize: bool = False) -> Tensor:
    """Optimal assignment of every ``[n, n]`` problem in a ROCm ``[B, n, n]`` cost batch (one wave per problem,
    Hungarian method; ``csrc/audio/lsa.hip``).  Returns int64 ``[B, n]``: the column of each row."""
    c = cost.detach()
    if c.dtype not in (torch.float32, torch.float64):
        c = c.float()
    out = torch.zeros(c.shape[0], c.shape[1], dtype=torch.int64, device=c.device)
    _ops().linear_sum_assignment(c.contiguous(), bool(maximize), out)
    return out


# ------------------------------------------------------------------------------------------------------- sync wire
NARROW_WIRE_DTYPES = (torch.uint8, torch.float16, torch.int32)  # wire codes 0 / 1 / 2 of csrc/comm/narrow_wire.hip


def narrow_encode(src: Tensor, code: int, world: int) -> Tensor:
    """An integer SUM bucket in the narrow wire dtype ``NARROW_WIRE_DTYPES[code]`` plus two check slots (too big for
    an exact ``world``-rank sum / negative), ``[n + 2]`` (``csrc/comm/narrow_wire.hip``)."""
    src = src.reshape(-1)
    if src.is_cuda:
        return _ops().narrow_encode(src.contiguous(), int(code), int(world))
    return _cpu.narrow_encode(src, int(code), int(world))


def static_gather_check(gathered: Tensor, word: Tensor, bit: int) -> None:
    """``word |= bit`` (on the device) when a rank's signature -- the last column of the gathered ``[W, L + 1]``
    static-shape bucket -- is not 1 (``csrc/comm/narrow_wire.hip``); CPU buckets are checked on the host."""
    if gathered.is_cuda:
        _ops().static_gather_check(gathered, word, int(bit))
    elif bool((gathered[:, -1] != 1).any()):
        word.bitwise_or_(int(bit))


def narrow_decode(wire: Tensor, n: int, out_dtype: torch.dtype, word: Optional[Tensor], bit: int) -> Tensor:
    """The summed wire widened back to ``out_dtype`` ``[n]``; ``word |= bit`` on the device when a check slot of the
    sum is set (the result is then not exact and the bucket must be re-sent wider)."""
    if wire.is_cuda:
        return _ops().narrow_decode(wire, int(n), out_dtype, word, int(bit))
    return _cpu.narrow_decode(wire, int(n), out_dtype, word, int(bit))
