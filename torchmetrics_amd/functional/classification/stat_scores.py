"""Stat scores (tp / fp / tn / fn / support) for binary, multiclass and multilabel tasks.

Semantics follow reference ``F/classification/stat_scores.py:25-818`` (thresholding with sigmoid auto-detection,
``ignore_index`` in/out of the label range, ``top_k``, ``average``, ``multidim_average``).  The computation is one
fused HIP kernel per update (``csrc/classification/stat_scores.hip``) instead of the reference's
validate(torch.unique) -> format -> one-hot/bincount -> algebra chain, and value validation is deferred on GPU.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.enums import ClassificationTask

# ------------------------------------------------------------------------------------------------ validation (args)


def _check_ignore_index(ignore_index: Optional[int]) -> None:
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")


def _check_multidim_average(multidim_average: str) -> None:
    allowed = ("global", "samplewise")
    if multidim_average not in allowed:
        raise ValueError(f"Expected argument `multidim_average` to be one of {allowed}, but got {multidim_average}")


def _binary_stat_scores_arg_validation(
    threshold: float = 0.5, multidim_average: str = "global", ignore_index: Optional[int] = None
) -> None:
    if not (isinstance(threshold, float) and (0 <= threshold <= 1)):
        raise ValueError(f"Expected argument `threshold` to be a float in the [0,1] range, but got {threshold}.")
    _check_multidim_average(multidim_average)
    _check_ignore_index(ignore_index)


def _multiclass_stat_scores_arg_validation(
    num_classes: int,
    top_k: int = 1,
    average: Optional[str] = "macro",
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
) -> None:
    if not isinstance(num_classes, int) or num_classes < 2:
        raise ValueError(f"Expected argument `num_classes` to be an integer larger than 1, but got {num_classes}")
    if not isinstance(top_k, int) and top_k < 1:
        raise ValueError(f"Expected argument `top_k` to be an integer larger than or equal to 1, but got {top_k}")
    if top_k > num_classes:
        raise ValueError(
            f"Expected argument `top_k` to be smaller or equal to `num_classes` but got {top_k} and {num_classes}"
        )
    allowed = ("micro", "macro", "weighted", "none", None)
    if average not in allowed:
        raise ValueError(f"Expected argument `average` to be one of {allowed}, but got {average}")
    _check_multidim_average(multidim_average)
    _check_ignore_index(ignore_index)


def _multilabel_stat_scores_arg_validation(
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[str] = "macro",
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
) -> None:
    if not isinstance(num_labels, int) or num_labels < 2:
        raise ValueError(f"Expected argument `num_labels` to be an integer larger than 1, but got {num_labels}")
    if not (isinstance(threshold, float) and (0 <= threshold <= 1)):
        raise ValueError(f"Expected argument `threshold` to be a float, but got {threshold}.")
    allowed = ("micro", "macro", "weighted", "none", None)
    if average not in allowed:
        raise ValueError(f"Expected argument `average` to be one of {allowed}, but got {average}")
    _check_multidim_average(multidim_average)
    _check_ignore_index(ignore_index)


# ---------------------------------------------------------------------------------------------- validation (shapes)
# Only host metadata is inspected here; value-range checks run inside the kernels (device flag on GPU).


def _binary_stat_scores_tensor_validation(
    preds: Tensor, target: Tensor, multidim_average: str = "global", ignore_index: Optional[int] = None
) -> None:
    _check_same_shape(preds, target)
    if multidim_average != "global" and preds.ndim < 2:
        raise ValueError("Expected input to be at least 2D when multidim_average is set to `samplewise`")


def _multiclass_stat_scores_tensor_validation(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
) -> None:
    pnd = preds.ndim
    if pnd == target.ndim + 1:
        if not preds.is_floating_point():
            raise ValueError("If `preds` have one dimension more than `target`, `preds` should be a float tensor.")
        if preds.shape[1] != num_classes:
            raise ValueError(
                "If `preds` have one dimension more than `target`, `preds.shape[1]` should be"
                " equal to number of classes."
            )
        if pnd > 2 and preds.shape[2:] != target.shape[1:]:
            raise ValueError(
                "If `preds` have one dimension more than `target`, the shape of `preds` should be"
                " (N, C, ...), and the shape of `target` should be (N, ...)."
            )
        if multidim_average != "global" and preds.ndim < 3:
            raise ValueError(
                "If `preds` have one dimension more than `target`, the shape of `preds` should "
                " at least 3D when multidim_average is set to `samplewise`"
            )
    elif pnd == target.ndim:
        if preds.shape != target.shape:
            raise ValueError(
                "The `preds` and `target` should have the same shape,",
                f" got `preds` with shape={preds.shape} and `target` with shape={target.shape}.",
            )
        if multidim_average != "global" and preds.ndim < 2:
            raise ValueError(
                "When `preds` and `target` have the same shape, the shape of `preds` should "
                " at least 2D when multidim_average is set to `samplewise`"
            )
    else:
        raise ValueError(
            "Either `preds` and `target` both should have the (same) shape (N, ...), or `target` should be (N, ...)"
            " and `preds` should be (N, C, ...)."
        )


def _multilabel_stat_scores_tensor_validation(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
) -> None:
    _check_same_shape(preds, target)
    if preds.shape[1] != num_labels:
        raise ValueError(
            "Expected both `target.shape[1]` and `preds.shape[1]` to be equal to the number of labels"
            f" but got {preds.shape[1]} and expected {num_labels}"
        )
    if multidim_average != "global" and preds.ndim < 3:
        raise ValueError("Expected input to be at least 3D when multidim_average is set to `samplewise`")


# ---------------------------------------------------------------------------------------------- fused statistics


def _as_target(target: Tensor) -> Tensor:
    if target.dtype in (torch.int64, torch.int32, torch.uint8, torch.bool):
        return target
    return target.long()


def _as_preds(preds: Tensor) -> Tensor:
    if preds.is_floating_point() or preds.dtype in (torch.int64, torch.int32, torch.uint8, torch.bool):
        return preds
    return preds.long()


class _StatWorkspace:
    """Reusable per-metric device buffers for the fused update (workspace re-zeroed by the finalize kernel)."""

    __slots__ = ("ws", "not_prob")

    def __init__(self) -> None:
        self.ws: Optional[Tensor] = None
        self.not_prob: Optional[Tensor] = None

    def get(self, numel: int, device: torch.device) -> Tuple[Tensor, Tensor]:
        if self.ws is None or self.ws.numel() != numel or self.ws.device != device:
            self.ws = torch.zeros(numel, dtype=torch.int64, device=device)
            # two words, double-buffered by update parity (csrc/classification/stat_scores.hip notprob_begin)
            self.not_prob = torch.zeros(2, dtype=torch.int32, device=device)
        return self.ws, self.not_prob  # type: ignore[return-value]


def _scratch_flag(device: torch.device) -> Tensor:
    """A fresh (zeroed) validation flag word, for callers that check it afterwards."""
    return torch.zeros(1, dtype=torch.int32, device=device)


_SINK: dict = {}


def _sink_flag(device: torch.device) -> Tensor:
    """A cached per-device flag word for callers that do not validate (no allocation per update)."""
    key = (device.type, device.index)
    buf = _SINK.get(key)
    if buf is None:
        buf = _SINK[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return buf


def _binary_like_stats(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float,
    multidim_average: str,
    ignore_index: Optional[int],
    flag: Optional[Tensor],
    out: Optional[Tuple[Tensor, Tensor, Tensor, Tensor]] = None,
    workspace: Optional[_StatWorkspace] = None,
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Run the fused binary/multilabel kernel; accumulate into ``out`` (global) or return fresh ``[G]`` tensors."""
    samplewise = multidim_average == "samplewise"
    dev = preds.device
    N = preds.shape[0] if preds.ndim else 1
    G = (N * num_labels) if samplewise else num_labels
    if workspace is not None and not samplewise:
        ws, not_prob = workspace.get(G * 7, dev)
    else:
        ws = torch.zeros(G * 7, dtype=torch.int64, device=dev)
        not_prob = torch.zeros(1, dtype=torch.int32, device=dev)
    if flag is None:
        flag = _sink_flag(dev)
    p = _as_preds(preds)
    t = _as_target(target)
    if p.ndim == 0:
        p, t = p.reshape(1), t.reshape(1)
    ops.bin_update(p, t, ws, flag, not_prob, num_labels, threshold, ignore_index, samplewise)
    if out is not None and not samplewise:
        ops.bin_stats_finalize(ws, not_prob, True, *out)
        return out
    res = tuple(torch.empty(G, dtype=torch.int64, device=dev) for _ in range(4))
    ops.bin_stats_finalize(ws, not_prob, False, *res)
    return res  # type: ignore[return-value]


def _multiclass_stats(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    top_k: int,
    micro: bool,
    multidim_average: str,
    ignore_index: Optional[int],
    flag: Optional[Tensor],
    out: Optional[Tuple[Tensor, Tensor, Tensor, Tensor]] = None,
    workspace: Optional[_StatWorkspace] = None,
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Fused multiclass stats. ``micro`` reduces over classes (state size 1; only for global, top_k == 1)."""
    samplewise = multidim_average == "samplewise"
    dev = preds.device
    t = _as_target(target)
    if t.ndim == 0:
        t = t.reshape(1)
        preds = preds.reshape(1, *preds.shape) if preds.ndim <= 1 else preds
    N = t.shape[0]
    fused_topk = top_k > 1 and preds.is_floating_point() and preds.ndim == 2 == t.ndim + 1
    if preds.is_floating_point() and preds.ndim == t.ndim + 1:
        p = preds
        if top_k > 1 and not fused_topk:
            p = preds.topk(top_k, dim=1).indices  # [N, K, ...] int64 labels
    else:
        p = _as_preds(preds)
    if flag is None:
        flag = _sink_flag(dev)
    C = num_classes
    G = N if samplewise else 1
    micro = micro and not samplewise
    if workspace is not None and not samplewise:
        ws, _ = workspace.get(G * (3 * C + 1), dev)
    else:
        ws = torch.zeros(G * (3 * C + 1), dtype=torch.int64, device=dev)
    # top_k > 1 on [N, C] scores: selection + histogram in one launch (topk.hip), else topk labels + mc_update
    if not (fused_topk and ops.mc_topk_update(preds, t, ws, flag, top_k, ignore_index, samplewise)):
        if fused_topk:
            p = preds.topk(top_k, dim=1).indices
        ops.mc_update(p.contiguous(), t.contiguous(), ws, flag, C, ignore_index, ops.MC_STATS, samplewise)
    if out is not None and not samplewise:
        ops.mc_stats_finalize(ws, C, micro, True, *out)
        return out
    size = G if micro else G * C
    res = tuple(torch.empty(size, dtype=torch.int64, device=dev) for _ in range(4))
    ops.mc_stats_finalize(ws, C, micro, False, *res)
    if samplewise:
        res = tuple(r.view(G, C) for r in res)
    return res  # type: ignore[return-value]


def _check_flag(flag: Tensor, ctx: object = None) -> None:
    """Raise a deferred validation error recorded by a kernel (one 4-byte D2H copy on GPU)."""
    from torchmetrics_amd.utils.validation import raise_for_code

    code = int(flag.item())
    if code:
        raise_for_code(code, ctx)


class _Ctx:
    def __init__(self, **kw: object) -> None:
        self.__dict__.update(kw)


def _binary_stat_scores_update(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """tp, fp, tn, fn for a binary batch (scalars for global, ``[N]`` for samplewise)."""
    flag = _scratch_flag(preds.device)
    N = preds.shape[0] if preds.ndim else 1
    tp, fp, tn, fn = _binary_like_stats(preds, target, 1, threshold, multidim_average, ignore_index, flag)
    if validate_args:
        _check_flag(flag)
    if multidim_average == "global":
        return tp.squeeze(), fp.squeeze(), tn.squeeze(), fn.squeeze()
    return tuple(x.view(N).squeeze() if N == 1 else x.view(N) for x in (tp, fp, tn, fn))  # type: ignore[return-value]


def _binary_stat_scores_compute(tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, multidim_average: str = "global") -> Tensor:
    return torch.stack([tp, fp, tn, fn, tp + fn], dim=0 if multidim_average == "global" else 1).squeeze()


def _multiclass_stat_scores_update(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    top_k: int = 1,
    average: Optional[str] = "macro",
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    flag = _scratch_flag(preds.device)
    micro = average == "micro" and top_k == 1 and multidim_average == "global"
    tp, fp, tn, fn = _multiclass_stats(preds, target, num_classes, top_k, micro, multidim_average, ignore_index, flag)
    if validate_args:
        _check_flag(flag, _Ctx(num_classes=num_classes))
    if micro:
        return tp.squeeze(), fp.squeeze(), tn.squeeze(), fn.squeeze()
    return tp, fp, tn, fn


def _multiclass_stat_scores_compute(
    tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, average: Optional[str] = "macro", multidim_average: str = "global"
) -> Tensor:
    if multidim_average == "global" and ops._RECORDER is not None:  # one task of the fused compute launch
        fused = ops.stat_scores_output(tp, fp, tn, fn, average)
        if fused is not None:
            return fused
    res = torch.stack([tp, fp, tn, fn, tp + fn], dim=-1)
    sum_dim = 0 if multidim_average == "global" else 1
    if average == "micro":
        return res.sum(sum_dim) if res.ndim > 1 else res
    if average == "macro":
        return res.float().mean(sum_dim)
    if average == "weighted":
        weight = tp + fn
        if multidim_average == "global":
            return (res * (weight / weight.sum()).reshape(*weight.shape, 1)).sum(sum_dim)
        return (res * (weight / weight.sum(-1, keepdim=True)).reshape(*weight.shape, 1)).sum(sum_dim)
    if average is None or average == "none":
        return res
    return None  # type: ignore[return-value]


def _multilabel_stat_scores_update(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    flag = _scratch_flag(preds.device)
    N = preds.shape[0]
    res = _binary_like_stats(preds, target, num_labels, threshold, multidim_average, ignore_index, flag)
    if validate_args:
        _check_flag(flag)
    if multidim_average == "samplewise":
        return tuple(r.view(N, num_labels) for r in res)  # type: ignore[return-value]
    return res


def _multilabel_stat_scores_compute(
    tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, average: Optional[str] = "macro", multidim_average: str = "global"
) -> Tensor:
    if multidim_average == "global" and ops._RECORDER is not None:  # one task of the fused compute launch
        fused = ops.stat_scores_output(tp, fp, tn, fn, average)
        if fused is not None:
            return fused
    res = torch.stack([tp, fp, tn, fn, tp + fn], dim=-1)
    sum_dim = 0 if multidim_average == "global" else 1
    if average == "micro":
        return res.sum(sum_dim)
    if average == "macro":
        return res.float().mean(sum_dim)
    if average == "weighted":
        w = tp + fn
        return (res * (w / w.sum()).reshape(*w.shape, 1)).sum(sum_dim)
    if average is None or average == "none":
        return res
    return None  # type: ignore[return-value]


# ------------------------------------------------------------------------------------------------------ public API


def binary_stat_scores(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[tp, fp, tn, fn, support]`` for binary tasks (``[N, 5]`` when ``multidim_average='samplewise'``)."""
    if validate_args:
        _binary_stat_scores_arg_validation(threshold, multidim_average, ignore_index)
        _binary_stat_scores_tensor_validation(preds, target, multidim_average, ignore_index)
    tp, fp, tn, fn = _binary_stat_scores_update(preds, target, threshold, multidim_average, ignore_index, validate_args)
    return _binary_stat_scores_compute(tp, fp, tn, fn, multidim_average)


def multiclass_stat_scores(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[str] = "macro",
    top_k: int = 1,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[tp, fp, tn, fn, support]`` per class (or reduced by ``average``) for multiclass tasks."""
    if validate_args:
        _multiclass_stat_scores_arg_validation(num_classes, top_k, average, multidim_average, ignore_index)
        _multiclass_stat_scores_tensor_validation(preds, target, num_classes, multidim_average, ignore_index)
    tp, fp, tn, fn = _multiclass_stat_scores_update(
        preds, target, num_classes, top_k, average, multidim_average, ignore_index, validate_args
    )
    return _multiclass_stat_scores_compute(tp, fp, tn, fn, average, multidim_average)


def multilabel_stat_scores(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[str] = "macro",
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[tp, fp, tn, fn, support]`` per label (or reduced by ``average``) for multilabel tasks."""
    if validate_args:
        _multilabel_stat_scores_arg_validation(num_labels, threshold, average, multidim_average, ignore_index)
        _multilabel_stat_scores_tensor_validation(preds, target, num_labels, multidim_average, ignore_index)
    tp, fp, tn, fn = _multilabel_stat_scores_update(
        preds, target, num_labels, threshold, multidim_average, ignore_index, validate_args
    )
    return _multilabel_stat_scores_compute(tp, fp, tn, fn, average, multidim_average)


def stat_scores(
    preds: Tensor,
    target: Tensor,
    task: str,
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[str] = "micro",
    multidim_average: str = "global",
    top_k: Optional[int] = 1,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Task-dispatching wrapper around the binary / multiclass / multilabel variants."""
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_stat_scores(preds, target, threshold, multidim_average, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        if not isinstance(top_k, int):
            raise ValueError(f"`top_k` is expected to be `int` but `{type(top_k)} was passed.`")
        return multiclass_stat_scores(
            preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args
        )
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_stat_scores(
            preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args
        )
    raise ValueError(f"Unsupported task `{task}`")
