"""Deferred, device-side input validation.

The reference validates value ranges eagerly in every ``update`` with host-synchronising reductions
(``len(torch.unique(target))`` ``F/classification/stat_scores.py:307``, ``torch.all(0<=preds<=1)`` ``:104``,
``nans.any()`` ``S/aggregation.py:90``).  On MI355X each of those is a full pipeline drain (~10-30 us each).

Here, the HIP kernels that consume the inputs also check them and ``atomicOr`` a bit into a per-metric int32 flag
word on the device.  The word is read once when the user calls ``compute()`` (or after every update with
``TORCHMETRICS_AMD_STRICT=1``), and the same exception type the reference would have raised is thrown.  CPU tensors
are validated eagerly (no sync cost on the host).
"""
import os
from typing import Any, Dict

STRICT = os.environ.get("TORCHMETRICS_AMD_STRICT", "0") == "1"

# bit layout shared with csrc/common/validation.h
TARGET_OUT_OF_RANGE = 1 << 0  # integer target outside [0, C) and != ignore_index
PREDS_OUT_OF_RANGE = 1 << 1  # integer preds outside [0, C)
TARGET_NOT_BINARY = 1 << 2  # binary/multilabel target not in {0, 1} (and != ignore_index)
PREDS_NOT_BINARY = 1 << 3  # binary/multilabel integer preds not in {0, 1}
PREDS_NAN = 1 << 4  # NaN in float preds where not allowed
VALUE_NAN = 1 << 5  # NaN in an aggregation input with nan_strategy='error'
NEG_VALUE = 1 << 6  # negative value where a non-negative one is required
VALUE_NAN_WARN = 1 << 7  # NaN dropped by an aggregator with nan_strategy='warn': a warning, not an error
ONESHOT_FAILED = 1 << 8  # the one-shot all-reduce of this metric's states timed out / was disowned by a peer
NARROW_RETRY = 1 << 9  # not an error: a narrow-wire bucket of this metric's sync overflowed, re-sync it wider

_MESSAGES: Dict[int, str] = {
    TARGET_OUT_OF_RANGE: "Detected more unique values in `target` than expected. Expected only {num_classes} values"
    " (in the range [0, {num_classes}) or equal to `ignore_index`).",
    PREDS_OUT_OF_RANGE: "Detected more unique values in `preds` than expected. Expected only {num_classes} values.",
    TARGET_NOT_BINARY: "Detected the following values in `target`: not all in [0, 1] but expected only the following"
    " values [0, 1] (or `ignore_index`).",
    PREDS_NOT_BINARY: "Detected the following values in `preds`: not all in [0, 1] but expected only the following"
    " values [0, 1] since `preds` is a label tensor.",
    PREDS_NAN: "Encountered `nan` values in `preds`.",
    VALUE_NAN: "Encountered `nan` values in tensor",
    NEG_VALUE: "Encountered negative values where non-negative values were expected.",
}


def raise_for_code(code: int, metric: Any = None) -> None:
    """Raise the first error encoded in ``code`` (warning bits are emitted as warnings; no raise if only those)."""
    code &= ~NARROW_RETRY  # handled by the owner's re-sync (Metric._raise_device_errors)
    if code & VALUE_NAN_WARN:
        from torchmetrics_amd.utilities.prints import rank_zero_warn

        rank_zero_warn("Encountered `nan` values in tensor. Will be removed.", UserWarning)
        code &= ~VALUE_NAN_WARN
        if not code:
            return
    if code & ONESHOT_FAILED:
        from torchmetrics_amd.parallel import oneshot

        oneshot.disable_all()  # every rank raises here, so every rank falls back to RCCL together
        raise RuntimeError(oneshot.failure_message())
    ctx = {"num_classes": getattr(metric, "num_classes", getattr(metric, "num_labels", "?"))}
    for bit, msg in _MESSAGES.items():
        if code & bit:
            if bit == VALUE_NAN:
                raise RuntimeError(msg.format(**ctx))
            raise RuntimeError(msg.format(**ctx))
    raise RuntimeError(f"Unknown device-side validation error code {code}")
