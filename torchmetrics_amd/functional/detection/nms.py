"""Non-maximum suppression (``torchvision.ops.nms`` / ``batched_nms`` contract), on the HIP bitmask kernel.

Not part of the reference (it evaluates given detections), provided because the usual pipeline runs NMS
right before :class:`~torchmetrics_amd.detection.MeanAveragePrecision` and BASELINE config #3 names it.  Ties in
score are broken by the lower index (stable order).
"""
from typing import Optional

from torch import Tensor

from torchmetrics_amd import ops


def nms(boxes: Tensor, scores: Tensor, iou_threshold: float) -> Tensor:
    """Indices (int64, descending score) of the ``[N, 4]`` xyxy boxes kept by greedy NMS at ``IoU > iou_threshold``."""
    _check(boxes, scores, None)
    return ops.nms(boxes, scores, iou_threshold)


def batched_nms(boxes: Tensor, scores: Tensor, idxs: Tensor, iou_threshold: float) -> Tensor:
    """Class-aware NMS: boxes only suppress boxes with the same ``idxs`` value (one pass, no coordinate offsets)."""
    _check(boxes, scores, idxs)
    return ops.nms(boxes, scores, iou_threshold, idxs)


def _check(boxes: Tensor, scores: Tensor, idxs: Optional[Tensor]) -> None:
    if boxes.ndim != 2 or boxes.shape[-1] != 4:
        raise ValueError(f"Expected `boxes` of shape [N, 4], got {tuple(boxes.shape)}")
    if scores.ndim != 1 or scores.shape[0] != boxes.shape[0]:
        raise ValueError(f"Expected `scores` of shape [{boxes.shape[0]}], got {tuple(scores.shape)}")
    if idxs is not None and (idxs.ndim != 1 or idxs.shape[0] != boxes.shape[0]):
        raise ValueError(f"Expected `idxs` of shape [{boxes.shape[0]}], got {tuple(idxs.shape)}")
