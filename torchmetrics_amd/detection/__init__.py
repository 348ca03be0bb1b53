"""Detection module metrics (parity: reference ``S/detection/__init__.py``)."""
from torchmetrics_amd.detection.iou import (
    CompleteIntersectionOverUnion,
    DistanceIntersectionOverUnion,
    GeneralizedIntersectionOverUnion,
    IntersectionOverUnion,
)
from torchmetrics_amd.detection.mean_ap import MeanAveragePrecision

__all__ = [
    "CompleteIntersectionOverUnion",
    "DistanceIntersectionOverUnion",
    "GeneralizedIntersectionOverUnion",
    "IntersectionOverUnion",
    "MeanAveragePrecision",
]
