"""Legacy result containers of the reference's pure-torch mAP (``S/detection/_mean_ap.py:73-110``).

``BaseMetricResults`` is a ``dict`` with attribute access; the three subclasses name the field groups of the COCO
summary.  The legacy ``MeanAveragePrecision`` of that module is the same metric as
:class:`torchmetrics_amd.detection.MeanAveragePrecision` here (one GPU COCO evaluator serves both).
"""
from typing import Any, List, Sequence, Union

import torch
from torch import Tensor

from torchmetrics_amd.detection.mean_ap import MeanAveragePrecision  # noqa: F401


class BaseMetricResults(dict):
    """``dict`` whose keys are also attributes (``AttributeError`` instead of ``KeyError`` for missing ones)."""

    def __getattr__(self, key: str) -> Tensor:
        if key in self:
            return self[key]
        raise AttributeError(f"No such attribute: {key}")

    def __setattr__(self, key: str, value: Tensor) -> None:
        self[key] = value

    def __delattr__(self, key: str) -> None:
        if key in self:
            del self[key]
            return
        raise AttributeError(f"No such attribute: {key}")


class MAPMetricResults(BaseMetricResults):
    """mAP fields of the COCO summary."""

    __slots__ = ("map", "map_50", "map_75", "map_small", "map_medium", "map_large", "classes")


class MARMetricResults(BaseMetricResults):
    """mAR fields of the COCO summary."""

    __slots__ = ("mar_1", "mar_10", "mar_100", "mar_small", "mar_medium", "mar_large")


class COCOMetricResults(BaseMetricResults):
    """All mAP / mAR fields of the COCO summary, plus the per-class vectors."""

    __slots__ = (
        "map", "map_50", "map_75", "map_small", "map_medium", "map_large", "mar_1", "mar_10", "mar_100",
        "mar_small", "mar_medium", "mar_large", "map_per_class", "mar_100_per_class",
    )



def _rle_counts(counts: Union[str, bytes, Sequence[int]]) -> List[int]:
    """COCO RLE run lengths; compressed strings use the COCO 6-bit / delta encoding of ``rleFrString``."""
    if not isinstance(counts, (str, bytes)):
        return [int(c) for c in counts]
    data = counts.encode() if isinstance(counts, str) else counts
    out: List[int] = []
    p = 0
    while p < len(data):
        x, k, more = 0, 0, True
        while more:
            c = data[p] - 48
            x |= (c & 0x1F) << (5 * k)
            more = bool(c & 0x20)
            p += 1
            k += 1
            if not more and (c & 0x10):
                x |= -1 << (5 * k)
        if len(out) > 2:
            x += out[-2]
        out.append(x)
    return out


def _as_mask(item: Any) -> Tensor:
    """A binary ``[H, W]`` mask from a tensor or an RLE ``(size, counts)`` tuple (column-major runs, 0s first)."""
    if isinstance(item, Tensor):
        return item.bool()
    size, counts = item[0], item[1]
    h, w = int(size[0]), int(size[1])
    runs = torch.tensor(_rle_counts(counts), dtype=torch.long)
    vals = torch.arange(runs.numel()) % 2 == 1
    flat = torch.repeat_interleave(vals, runs)
    flat = torch.cat([flat, flat.new_zeros(h * w - flat.numel())]) if flat.numel() < h * w else flat[: h * w]
    return flat.reshape(w, h).t()


def compute_area(inputs: List[Any], iou_type: str = "bbox") -> Tensor:
    """Areas of boxes (``[4]`` xyxy rows) or of masks (tensors or RLE ``(size, counts)`` tuples)."""
    if len(inputs) == 0:
        return Tensor([])
    if iou_type == "bbox":
        b = torch.stack(list(inputs))
        return (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    if iou_type == "segm":
        return torch.tensor([float(_as_mask(i).sum()) for i in inputs], dtype=torch.float64)
    raise Exception(f"IOU type {iou_type} is not supported")  # noqa: TRY002 - reference contract


def compute_iou(det: List[Any], gt: List[Any], iou_type: str = "bbox") -> Tensor:
    """IoU matrix between detections and ground truths (boxes go through the HIP box kernel on ROCm tensors)."""
    if iou_type == "bbox":
        from torchmetrics_amd.functional.detection import intersection_over_union

        return intersection_over_union(torch.stack(list(det)), torch.stack(list(gt)), aggregate=False)
    if iou_type == "segm":
        d = torch.stack([_as_mask(i).reshape(-1) for i in det]).double()
        g = torch.stack([_as_mask(i).reshape(-1) for i in gt]).double()
        inter = d @ g.t()
        union = d.sum(1, keepdim=True) + g.sum(1)[None, :] - inter
        return torch.where(union > 0, inter / union, torch.zeros_like(inter))
    raise Exception(f"IOU type {iou_type} is not supported")  # noqa: TRY002 - reference contract
