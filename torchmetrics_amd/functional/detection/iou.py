"""IoU / GIoU / DIoU / CIoU between box sets (reference ``F/detection/{iou,giou,diou,ciou}.py``).

The reference calls the torchvision box ops; here all four run through one HIP kernel
(``csrc/detection/box_ops.hip``, ``ops.box_pairwise``) and ``aggregate=True`` evaluates only the aligned pairs
instead of the full ``N x M`` matrix.
"""
from typing import Optional

import torch
from torch import Tensor

from torchmetrics_amd import ops


def _box_update(preds: Tensor, target: Tensor, op: int, iou_threshold: Optional[float],
                replacement_val: float = 0) -> Tensor:
    iou = ops.box_pairwise(preds, target, op)
    if iou_threshold is not None:
        iou = torch.where(iou < iou_threshold, torch.full_like(iou, replacement_val), iou)
    return iou


def _box_compute(iou: Tensor, aggregate: bool = True) -> Tensor:
    if not aggregate:
        return iou
    return iou.diag().mean() if iou.numel() > 0 else torch.tensor(0.0, device=iou.device)


def _box_metric(preds: Tensor, target: Tensor, op: int, iou_threshold: Optional[float], replacement_val: float,
                aggregate: bool) -> Tensor:
    if aggregate and iou_threshold is None:
        n = min(preds.shape[0], target.shape[0])
        if n == 0:
            return torch.tensor(0.0, device=preds.device)
        return ops.box_pairwise(preds[:n], target[:n], op, aligned=True).mean()
    return _box_compute(_box_update(preds, target, op, iou_threshold, replacement_val), aggregate)


def _iou_update(preds: Tensor, target: Tensor, iou_threshold: Optional[float], replacement_val: float = 0) -> Tensor:
    return _box_update(preds, target, ops.BOX_IOU, iou_threshold, replacement_val)


def _giou_update(preds: Tensor, target: Tensor, iou_threshold: Optional[float], replacement_val: float = 0) -> Tensor:
    return _box_update(preds, target, ops.BOX_GIOU, iou_threshold, replacement_val)


def _diou_update(preds: Tensor, target: Tensor, iou_threshold: Optional[float], replacement_val: float = 0) -> Tensor:
    return _box_update(preds, target, ops.BOX_DIOU, iou_threshold, replacement_val)


def _ciou_update(preds: Tensor, target: Tensor, iou_threshold: Optional[float], replacement_val: float = 0) -> Tensor:
    return _box_update(preds, target, ops.BOX_CIOU, iou_threshold, replacement_val)


_iou_compute = _giou_compute = _diou_compute = _ciou_compute = _box_compute


def intersection_over_union(preds: Tensor, target: Tensor, iou_threshold: Optional[float] = None,
                            replacement_val: float = 0, aggregate: bool = True) -> Tensor:
    """IoU of xyxy boxes: matrix ``[N, M]`` or (``aggregate``) the mean over aligned pairs."""
    return _box_metric(preds, target, ops.BOX_IOU, iou_threshold, replacement_val, aggregate)


def generalized_intersection_over_union(preds: Tensor, target: Tensor, iou_threshold: Optional[float] = None,
                                        replacement_val: float = 0, aggregate: bool = True) -> Tensor:
    """Generalised IoU (IoU minus the empty fraction of the enclosing box)."""
    return _box_metric(preds, target, ops.BOX_GIOU, iou_threshold, replacement_val, aggregate)


def distance_intersection_over_union(preds: Tensor, target: Tensor, iou_threshold: Optional[float] = None,
                                     replacement_val: float = 0, aggregate: bool = True) -> Tensor:
    """Distance IoU (IoU minus normalised centre distance)."""
    return _box_metric(preds, target, ops.BOX_DIOU, iou_threshold, replacement_val, aggregate)


def complete_intersection_over_union(preds: Tensor, target: Tensor, iou_threshold: Optional[float] = None,
                                     replacement_val: float = 0, aggregate: bool = True) -> Tensor:
    """Complete IoU (DIoU plus aspect-ratio consistency term)."""
    return _box_metric(preds, target, ops.BOX_CIOU, iou_threshold, replacement_val, aggregate)
