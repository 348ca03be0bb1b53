"""IoU-family detection module metrics (parity: reference ``S/detection/{iou,giou,diou,ciou}.py``)."""
from typing import Any, Dict, List, Optional

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.detection.helpers import _fix_empty_tensors, _input_validator, box_convert
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import dim_zero_cat


class IntersectionOverUnion(Metric):
    """Mean IoU of all (prediction, target) box pairs (of matching labels by default) over all images."""

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = True
    plot_lower_bound: Optional[float] = None
    plot_upper_bound: Optional[float] = None
    groundtruth_labels: List[Tensor]
    iou_matrix: List[Tensor]
    _iou_type: str = "iou"
    _op: int = ops.BOX_IOU
    _invalid_val: float = -1.0

    def __init__(self, box_format: str = "xyxy", iou_threshold: Optional[float] = None, class_metrics: bool = False,
                 respect_labels: bool = True, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        allowed = ("xyxy", "xywh", "cxcywh")
        if box_format not in allowed:
            raise ValueError(f"Expected argument `box_format` to be one of {allowed} but got {box_format}")
        self.box_format = box_format
        self.iou_threshold = iou_threshold
        if not isinstance(class_metrics, bool):
            raise ValueError("Expected argument `class_metrics` to be a boolean")
        self.class_metrics = class_metrics
        if not isinstance(respect_labels, bool):
            raise ValueError("Expected argument `respect_labels` to be a boolean")
        self.respect_labels = respect_labels
        self.add_state("groundtruth_labels", default=[], dist_reduce_fx=None)
        self.add_state("iou_matrix", default=[], dist_reduce_fx=None)

    def _safe_boxes(self, boxes: Tensor) -> Tensor:
        boxes = _fix_empty_tensors(boxes)
        if boxes.numel() > 0:
            boxes = box_convert(boxes, in_fmt=self.box_format, out_fmt="xyxy")
        return boxes.reshape(-1, 4) if boxes.numel() else boxes.new_zeros(0, 4)

    def update(self, preds: List[Dict[str, Tensor]], target: List[Dict[str, Tensor]]) -> None:
        _input_validator(preds, target, ignore_score=True)
        for p, t in zip(preds, target):
            det, gt = self._safe_boxes(p["boxes"]), self._safe_boxes(t["boxes"])
            self.groundtruth_labels.append(t["labels"])
            mat = ops.box_pairwise(det, gt, self._op)
            if self.iou_threshold is not None:
                mat = torch.where(mat < self.iou_threshold, torch.full_like(mat, self._invalid_val), mat)
            if self.respect_labels:
                same = p["labels"].unsqueeze(1) == t["labels"].unsqueeze(0)
                mat = torch.where(same, mat, torch.full_like(mat, self._invalid_val))
            self.iou_matrix.append(mat)

    def compute(self) -> dict:
        valid = [m[m != self._invalid_val] for m in self.iou_matrix]
        score = torch.cat(valid, 0).mean() if valid else torch.tensor(float("nan"))
        results: Dict[str, Tensor] = {f"{self._iou_type}": score}
        if self.class_metrics:
            gt_labels = dim_zero_cat(self.groundtruth_labels) if self.groundtruth_labels else torch.zeros(0)
            for cl in (gt_labels.unique().tolist() if len(gt_labels) > 0 else []):
                tot, cnt = torch.zeros_like(score), torch.zeros_like(score)
                for mat, lab in zip(self.iou_matrix, self.groundtruth_labels):
                    s = mat[:, lab == cl]
                    keep = s != self._invalid_val
                    tot = tot + s[keep].sum()
                    cnt = cnt + keep.sum()
                results[f"{self._iou_type}/cl_{cl}"] = tot / cnt
        return results


class GeneralizedIntersectionOverUnion(IntersectionOverUnion):
    """Mean generalised IoU (GIoU)."""

    plot_lower_bound: Optional[float] = None
    _iou_type: str = "giou"
    _op: int = ops.BOX_GIOU
    _invalid_val: float = -1.0


class DistanceIntersectionOverUnion(IntersectionOverUnion):
    """Mean distance IoU (DIoU)."""

    plot_lower_bound: Optional[float] = None
    _iou_type: str = "diou"
    _op: int = ops.BOX_DIOU
    _invalid_val: float = -1.0


class CompleteIntersectionOverUnion(IntersectionOverUnion):
    """Mean complete IoU (CIoU)."""

    plot_lower_bound: Optional[float] = None
    _iou_type: str = "ciou"
    _op: int = ops.BOX_CIOU
    _invalid_val: float = -2.0
