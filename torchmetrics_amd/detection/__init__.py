"""Detection module metrics (parity: reference ``S/detection/__init__.py``)."""
from torchmetrics_amd.detection.iou import (
    CompleteIntersectionOverUnion,
    DistanceIntersectionOverUnion,
    GeneralizedIntersectionOverUnion,
    IntersectionOverUnion,
)
from torchmetrics_amd.detection.mean_ap import MeanAveragePrecision
from torchmetrics_amd.detection.panoptic_qualities import ModifiedPanopticQuality, PanopticQuality

__all__ = [
    "CompleteIntersectionOverUnion",
    "DistanceIntersectionOverUnion",
    "GeneralizedIntersectionOverUnion",
    "IntersectionOverUnion",
    "MeanAveragePrecision",
    "ModifiedPanopticQuality",
    "PanopticQuality",
]
