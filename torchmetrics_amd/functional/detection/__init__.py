"""Functional detection metrics (parity: reference ``F/detection/__init__.py``)."""
from torchmetrics_amd.functional.detection.iou import (
    complete_intersection_over_union,
    distance_intersection_over_union,
    generalized_intersection_over_union,
    intersection_over_union,
)
from torchmetrics_amd.functional.detection.nms import batched_nms, nms
from torchmetrics_amd.functional.detection.panoptic_qualities import modified_panoptic_quality, panoptic_quality

__all__ = [k for k in dir() if not k.startswith("_")]
