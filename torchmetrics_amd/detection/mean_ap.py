"""COCO mean average precision / recall (parity: reference ``S/detection/mean_ap.py:76-1048``).

The reference converts every state to COCO json-like dicts on the host and runs pycocotools / faster-coco-eval.
Here the same COCO protocol (IoU thresholds, 101 recall thresholds, max-detections 1/10/100, small / medium / large
areas, crowd handling, macro / micro averaging, per-class numbers, extended summary) is evaluated on the device by
:mod:`torchmetrics_amd.detection._coco_eval` (HIP greedy matcher + batched accumulation); no pycocotools needed.

Deliberate difference: ``iou_type="segm"`` states keep the binary masks as tensors (the reference keeps RLE tuples).
"""
import contextlib
import io
import json
from typing import Any, ClassVar, Dict, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd.detection._coco_eval import coco_evaluate, coco_summarize, per_class_stats
from torchmetrics_amd.detection.helpers import _fix_empty_tensors, _input_validator, _validate_iou_type_arg, box_convert
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.prints import rank_zero_warn


class MeanAveragePrecision(Metric):
    """COCO-style mAP / mAR for object detection (``bbox`` and/or ``segm``)."""

    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    detection_box: List[Tensor]
    detection_mask: List[Tensor]
    detection_scores: List[Tensor]
    detection_labels: List[Tensor]
    groundtruth_box: List[Tensor]
    groundtruth_mask: List[Tensor]
    groundtruth_labels: List[Tensor]
    groundtruth_crowds: List[Tensor]
    groundtruth_area: List[Tensor]

    warn_on_many_detections: bool = True
    __jit_unused_properties__: ClassVar[List[str]] = [
        "is_differentiable", "higher_is_better", "plot_lower_bound", "plot_upper_bound", "plot_legend_name",
        "metric_state", "_update_called",
    ]

    def __init__(
        self,
        box_format: Literal["xyxy", "xywh", "cxcywh"] = "xyxy",
        iou_type: Union[Literal["bbox", "segm"], Tuple[str]] = "bbox",
        iou_thresholds: Optional[List[float]] = None,
        rec_thresholds: Optional[List[float]] = None,
        max_detection_thresholds: Optional[List[int]] = None,
        class_metrics: bool = False,
        extended_summary: bool = False,
        average: Literal["macro", "micro"] = "macro",
        backend: Literal["pycocotools", "faster_coco_eval"] = "pycocotools",
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        allowed_box_formats = ("xyxy", "xywh", "cxcywh")
        if box_format not in allowed_box_formats:
            raise ValueError(f"Expected argument `box_format` to be one of {allowed_box_formats} but got {box_format}")
        self.box_format = box_format
        self.iou_type = _validate_iou_type_arg(iou_type)
        if iou_thresholds is not None and not isinstance(iou_thresholds, list):
            raise ValueError(
                f"Expected argument `iou_thresholds` to either be `None` or a list of floats but got {iou_thresholds}"
            )
        self.iou_thresholds = iou_thresholds or torch.linspace(0.5, 0.95, round((0.95 - 0.5) / 0.05) + 1).tolist()
        if rec_thresholds is not None and not isinstance(rec_thresholds, list):
            raise ValueError(
                f"Expected argument `rec_thresholds` to either be `None` or a list of floats but got {rec_thresholds}"
            )
        self.rec_thresholds = rec_thresholds or torch.linspace(0.0, 1.00, round(1.00 / 0.01) + 1).tolist()
        if max_detection_thresholds is not None and not isinstance(max_detection_thresholds, list):
            raise ValueError(
                f"Expected argument `max_detection_thresholds` to either be `None` or a list of ints"
                f" but got {max_detection_thresholds}"
            )
        if max_detection_thresholds is not None and len(max_detection_thresholds) != 3:
            raise ValueError(
                "When providing a list of max detection thresholds it should have length 3."
                f" Got value {len(max_detection_thresholds)}"
            )
        self.max_detection_thresholds = sorted(int(x) for x in (max_detection_thresholds or [1, 10, 100]))
        if not isinstance(class_metrics, bool):
            raise ValueError("Expected argument `class_metrics` to be a boolean")
        self.class_metrics = class_metrics
        if not isinstance(extended_summary, bool):
            raise ValueError("Expected argument `extended_summary` to be a boolean")
        self.extended_summary = extended_summary
        if average not in ("macro", "micro"):
            raise ValueError(f"Expected argument `average` to be one of ('macro', 'micro') but got {average}")
        self.average = average
        if backend not in ("pycocotools", "faster_coco_eval"):
            raise ValueError(
                f"Expected argument `backend` to be one of ('pycocotools', 'faster_coco_eval') but got {backend}"
            )
        # both names select the one native evaluator; kept for API compatibility
        self.backend = backend
        for name in ("detection_box", "detection_mask", "detection_scores", "detection_labels", "groundtruth_box",
                     "groundtruth_mask", "groundtruth_labels", "groundtruth_crowds", "groundtruth_area"):
            self.add_state(name, default=[], dist_reduce_fx=None)

    # ------------------------------------------------------------------------------------------------ update
    def update(self, preds: List[Dict[str, Tensor]], target: List[Dict[str, Tensor]]) -> None:
        _input_validator(preds, target, iou_type=self.iou_type)
        # per-image work is batched over the whole call: one box conversion for all images (the reference converts
        # image by image, ~4 launches each) and one zero tensor for all missing `iscrowd` / `area` entries
        det_boxes = self._convert_boxes([item["boxes"] for item in preds]) if "bbox" in self.iou_type else None
        gt_boxes = self._convert_boxes([item["boxes"] for item in target]) if "bbox" in self.iou_type else None
        limit = self.max_detection_thresholds[-1]
        for i, item in enumerate(preds):
            if det_boxes is not None:
                self.detection_box.append(det_boxes[i])
            if "segm" in self.iou_type:
                self.detection_mask.append(item["masks"].bool())
            if self.warn_on_many_detections and len(item["labels"]) > limit:
                _warning_on_too_many_detections(limit)
            self.detection_labels.append(item["labels"])
            self.detection_scores.append(item["scores"])
        crowds = self._defaults_for(target, "iscrowd")
        areas = self._defaults_for(target, "area")
        for i, item in enumerate(target):
            if gt_boxes is not None:
                self.groundtruth_box.append(gt_boxes[i])
            if "segm" in self.iou_type:
                self.groundtruth_mask.append(item["masks"].bool())
            self.groundtruth_labels.append(item["labels"])
            self.groundtruth_crowds.append(item["iscrowd"] if "iscrowd" in item else crowds[i])
            self.groundtruth_area.append(item["area"] if "area" in item else areas[i])

    def _convert_boxes(self, boxes: List[Tensor]) -> List[Tensor]:
        """``box_convert(..., out_fmt="xywh")`` of every non-empty ``[n, 4]`` tensor, as one batched conversion."""
        fixed = [_fix_empty_tensors(b) for b in boxes]
        if len(fixed) > 1 and all(b.ndim == 2 and b.shape[-1] == 4 for b in fixed) and \
                len({(b.device, b.dtype) for b in fixed}) == 1:
            sizes = [b.shape[0] for b in fixed]
            return list(torch.split(box_convert(torch.cat(fixed), in_fmt=self.box_format, out_fmt="xywh"), sizes))
        return [box_convert(b, in_fmt=self.box_format, out_fmt="xywh") if b.numel() > 0 else b for b in fixed]

    @staticmethod
    def _defaults_for(target: List[Dict[str, Tensor]], key: str) -> List[Optional[Tensor]]:
        """Zero ``[n_i]`` tensors (``zeros_like(labels)``) for the images without ``key``, carved from one allocation."""
        missing = [i for i, t in enumerate(target) if key not in t]
        out: List[Optional[Tensor]] = [None] * len(target)
        if not missing:
            return out
        labels = [target[i]["labels"] for i in missing]
        if len({(t.device, t.dtype) for t in labels}) == 1 and all(t.ndim == 1 for t in labels):
            parts = torch.split(torch.zeros(sum(t.numel() for t in labels), dtype=labels[0].dtype,
                                            device=labels[0].device), [t.numel() for t in labels])
        else:
            parts = [torch.zeros_like(t) for t in labels]
        for i, z in zip(missing, parts):
            out[i] = z
        return out

    # ----------------------------------------------------------------------------------------------- compute
    def _get_classes(self) -> List[int]:
        if len(self.detection_labels) > 0 or len(self.groundtruth_labels) > 0:
            return torch.cat(self.detection_labels + self.groundtruth_labels).unique().cpu().tolist()
        return []

    def _state_device(self) -> torch.device:
        for lst in (self.detection_labels, self.groundtruth_labels):
            if len(lst):
                return lst[0].device
        return self.device

    def _evaluate(self, i_type: str, micro: bool) -> Dict[str, Tensor]:
        dev = self._state_device()
        classes = torch.tensor(self._get_classes(), dtype=torch.long, device=dev)
        relabel = (lambda xs: [torch.zeros_like(x) for x in xs]) if micro else (lambda xs: list(xs))
        n = len(self.detection_labels)
        boxes_ok = i_type == "bbox"
        empty_box = torch.zeros(0, 4, device=dev)
        return coco_evaluate(
            det_boxes=[b.reshape(-1, 4) for b in self.detection_box] if boxes_ok else [empty_box] * n,
            det_scores=self.detection_scores,
            det_labels=relabel(self.detection_labels),
            gt_boxes=[b.reshape(-1, 4) for b in self.groundtruth_box] if boxes_ok else [empty_box] * n,
            gt_labels=relabel(self.groundtruth_labels),
            gt_crowds=self.groundtruth_crowds,
            # with both iou types the reference keeps the ground-truth area of the mask for the bbox evaluation too
            gt_areas=self.groundtruth_area if len(self.iou_type) == 1 else [
                torch.where(a > 0, a.double(), m.flatten(1).sum(1).double())
                for a, m in zip(self.groundtruth_area, self.groundtruth_mask)],
            iou_thresholds=self.iou_thresholds,
            rec_thresholds=self.rec_thresholds,
            max_dets=self.max_detection_thresholds,
            classes=classes,
            det_masks=None if boxes_ok else self.detection_mask,
            gt_masks=None if boxes_ok else self.groundtruth_mask,
        )

    def compute(self) -> dict:
        result: Dict[str, Tensor] = {}
        mdt = self.max_detection_thresholds
        for i_type in self.iou_type:
            prefix = "" if len(self.iou_type) == 1 else f"{i_type}_"
            ev = self._evaluate(i_type, micro=self.average == "micro")
            stats = coco_summarize(ev, self.iou_thresholds, mdt).to(torch.float32).cpu()
            names = ["map", "map_50", "map_75", "map_small", "map_medium", "map_large", f"mar_{mdt[0]}",
                     f"mar_{mdt[1]}", f"mar_{mdt[2]}", "mar_small", "mar_medium", "mar_large"]
            result.update({f"{prefix}{k}": stats[i] for i, k in enumerate(names)})
            if self.extended_summary:
                result.update({
                    f"{prefix}ious": self._ious(i_type),
                    f"{prefix}precision": ev["precision"].float().cpu(),
                    f"{prefix}recall": ev["recall"].float().cpu(),
                    f"{prefix}scores": ev["scores"].float().cpu(),
                })
            if self.class_metrics:
                ev_cls = self._evaluate(i_type, micro=False) if self.average == "micro" else ev
                mp, mr = per_class_stats(ev_cls)
                map_pc, mar_pc = mp.to(torch.float32).cpu(), mr.to(torch.float32).cpu()
            else:
                map_pc = torch.tensor([-1.0], dtype=torch.float32)
                mar_pc = torch.tensor([-1.0], dtype=torch.float32)
            result.update({f"{prefix}map_per_class": map_pc, f"{prefix}mar_{mdt[-1]}_per_class": mar_pc})
        result.update({"classes": torch.tensor(self._get_classes(), dtype=torch.int32)})
        return result

    def _ious(self, i_type: str) -> Dict[Tuple[int, int], Tensor]:
        """Per (image, class) IoU matrices: detections in score order (max-dets truncated) x ground truths."""
        out: Dict[Tuple[int, int], Tensor] = {}
        classes = self._get_classes()
        for img in range(len(self.detection_labels)):
            for cls in classes:
                dl, gl = self.detection_labels[img] == cls, self.groundtruth_labels[img] == cls
                if not bool(dl.any()) and not bool(gl.any()):
                    continue
                scores = self.detection_scores[img][dl]
                order = torch.argsort(-scores, stable=True)[: self.max_detection_thresholds[-1]]
                if i_type == "bbox":
                    d = self.detection_box[img].reshape(-1, 4)[dl][order]
                    g = self.groundtruth_box[img].reshape(-1, 4)[gl]
                    crowd = self.groundtruth_crowds[img][gl].bool()
                    mat = _coco_iou_matrix(d.double(), g.double(), crowd).float().cpu()
                else:
                    dm = self.detection_mask[img][dl][order].flatten(1).float()
                    gm = self.groundtruth_mask[img][gl].flatten(1).float()
                    inter = dm @ gm.T
                    crowd = self.groundtruth_crowds[img][gl].bool()
                    union = torch.where(crowd[None], dm.sum(1)[:, None], dm.sum(1)[:, None] + gm.sum(1)[None] - inter)
                    mat = (inter / union.clamp(min=1e-12)).float().cpu()
                out[(img, cls)] = mat
        return out

    # ---------------------------------------------------------------------------------------- COCO interop
    def tm_to_coco(self, name: str = "tm_map_input") -> None:
        """Write the accumulated boxes as COCO json files ``{name}_preds.json`` / ``{name}_target.json``."""
        def fmt(labels, boxes, scores=None, crowds=None, areas=None):
            images, anns, aid = [], [], 1
            for img, lab in enumerate(labels):
                images.append({"id": img})
                b = boxes[img].reshape(-1, 4).cpu().tolist() if boxes else []
                for k, label in enumerate(lab.cpu().tolist()):
                    area = float(areas[img][k]) if areas is not None and float(areas[img][k]) > 0 else (
                        b[k][2] * b[k][3] if b else 0.0)
                    ann = {"id": aid, "image_id": img, "area": area, "category_id": int(label),
                           "iscrowd": int(crowds[img][k]) if crowds is not None else 0}
                    if b:
                        ann["bbox"] = b[k]
                    if scores is not None:
                        ann["score"] = float(scores[img][k])
                    anns.append(ann)
                    aid += 1
            cats = [{"id": i, "name": str(i)} for i in self._get_classes()]
            return {"images": images, "annotations": anns, "categories": cats}

        target = fmt(self.groundtruth_labels, self.groundtruth_box, crowds=self.groundtruth_crowds,
                     areas=self.groundtruth_area)
        preds = fmt(self.detection_labels, self.detection_box, scores=self.detection_scores)
        with open(f"{name}_preds.json", "w") as f:
            f.write(json.dumps(preds["annotations"], indent=4))
        with open(f"{name}_target.json", "w") as f:
            f.write(json.dumps(target, indent=4))

    @staticmethod
    def coco_to_tm(
        coco_preds: str,
        coco_target: str,
        iou_type: Union[Literal["bbox", "segm"], List[str]] = "bbox",
        backend: Literal["pycocotools", "faster_coco_eval"] = "pycocotools",
    ) -> Tuple[List[Dict[str, Tensor]], List[Dict[str, Tensor]]]:
        """Read COCO json (target dataset + prediction list) into the ``update`` input format (bbox)."""
        iou_type = _validate_iou_type_arg(iou_type)
        if "segm" in iou_type:
            raise NotImplementedError("coco_to_tm: RLE / polygon decoding of `segm` annotations is not supported")
        with open(coco_target) as f:
            gt = json.load(f)
        with open(coco_preds) as f:
            dt = json.load(f)
        order = [img["id"] for img in gt.get("images", [])]
        for ann in gt["annotations"]:
            if ann["image_id"] not in order:
                order.append(ann["image_id"])
        target = {i: {"boxes": [], "labels": [], "iscrowd": [], "area": []} for i in order}
        for ann in gt["annotations"]:
            t = target[ann["image_id"]]
            t["boxes"].append(ann["bbox"])
            t["labels"].append(ann["category_id"])
            t["iscrowd"].append(ann.get("iscrowd", 0))
            t["area"].append(ann.get("area", 0.0))
        preds = {i: {"boxes": [], "labels": [], "scores": []} for i in order}
        for ann in dt:
            p = preds.setdefault(ann["image_id"], {"boxes": [], "labels": [], "scores": []})
            p["boxes"].append(ann["bbox"])
            p["labels"].append(ann["category_id"])
            p["scores"].append(ann["score"])
        bp, bt = [], []
        for key in order:
            p, t = preds[key], target[key]
            bp.append({"boxes": torch.tensor(p["boxes"], dtype=torch.float32).reshape(-1, 4),
                       "scores": torch.tensor(p["scores"], dtype=torch.float32),
                       "labels": torch.tensor(p["labels"], dtype=torch.int32)})
            bt.append({"boxes": torch.tensor(t["boxes"], dtype=torch.float32).reshape(-1, 4),
                       "labels": torch.tensor(t["labels"], dtype=torch.int32),
                       "iscrowd": torch.tensor(t["iscrowd"], dtype=torch.int32),
                       "area": torch.tensor(t["area"], dtype=torch.float32)})
        return bp, bt


def _coco_iou_matrix(d: Tensor, g: Tensor, crowd: Tensor) -> Tensor:
    """COCO (pycocotools ``maskUtils.iou``) box IoU of xywh boxes ``[n, 4] x [m, 4]``; crowd columns divide by the
    detection area."""
    x1 = torch.maximum(d[:, None, 0], g[None, :, 0])
    y1 = torch.maximum(d[:, None, 1], g[None, :, 1])
    x2 = torch.minimum(d[:, None, 0] + d[:, None, 2], g[None, :, 0] + g[None, :, 2])
    y2 = torch.minimum(d[:, None, 1] + d[:, None, 3], g[None, :, 1] + g[None, :, 3])
    w, h = x2 - x1, y2 - y1
    inter = torch.where((w > 0) & (h > 0), w * h, torch.zeros_like(w))
    da = (d[:, 2] * d[:, 3])[:, None]
    union = torch.where(crowd[None, :], da, da + (g[:, 2] * g[:, 3])[None, :] - inter)
    return torch.where(inter > 0, inter / union, torch.zeros_like(inter))


def _warning_on_too_many_detections(limit: int) -> None:
    rank_zero_warn(
        f"Encountered more than {limit} detections in a single image. This means that certain detections with the"
        " lowest scores will be ignored, that may have an undesirable impact on performance. Please consider adjusting"
        " the `max_detection_threshold` to suit your use case. To disable this warning, set attribute class"
        " `warn_on_many_detections=False`, after initializing the metric.",
        UserWarning,
    )
