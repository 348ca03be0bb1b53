"""COCO mean average precision / recall (parity: reference ``S/detection/mean_ap.py:76-1048``).

The reference converts every state to COCO json-like dicts on the host and runs pycocotools / faster-coco-eval.
Here the same COCO protocol (IoU thresholds, 101 recall thresholds, max-detections 1/10/100, small / medium / large
areas, crowd handling, macro / micro averaging, per-class numbers, extended summary) is evaluated on the device by
:mod:`torchmetrics_amd.detection._coco_eval` (HIP greedy matcher + batched accumulation); no pycocotools needed.

``iou_type="segm"``: masks are run-length encoded on the device in ``update`` (``csrc/detection/rle.hip``; the
reference encodes on the host with pycocotools, ``S/detection/mean_ap.py:825-829``) and kept as one int32 pack per
image -- ordinary tensor list states, so the sync engine gathers them (the reference needs ``all_gather_object``,
``:1007-1038``) -- and mask IoUs come from the runs (``ops.rle_iou``), never from dense ``[n, H, W]`` masks.
"""
import contextlib
import io
import json
from collections.abc import Mapping
from typing import Any, ClassVar, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.detection import _rle
from torchmetrics_amd.detection._coco_eval import (
    Packed,
    cat_states,
    coco_evaluate,
    coco_summarize,
    summarize_all,
    image_sizes,
    per_class_stats,
)
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
    _BOX_STATES = ("detection_box", "groundtruth_box")
    # the per-image tensor lists cross the sync engine as flat buffers (Metric._packed_sync_plan)
    _packed_sync_states = ("detection_box", "detection_scores", "detection_labels", "groundtruth_box",
                           "groundtruth_labels", "groundtruth_crowds", "groundtruth_area")

    def update(self, preds: List[Dict[str, Tensor]], target: List[Dict[str, Tensor]]) -> None:
        """Append the batch's images.  The whole batch is a handful of launches: per state ONE ``cat`` of all images
        stored as one chunk (``Metric._append_chunk``: per-image views are only built if something reads the list),
        one box conversion, one zero tensor for the missing ``iscrowd`` / ``area`` entries.  The reference appends
        9 tensors per image and converts boxes image by image (``S/detection/mean_ap.py:470-511``)."""
        if self._native_pack(preds, target):
            return
        _input_validator(preds, target, iou_type=self.iou_type)
        if not preds:
            return
        if self.warn_on_many_detections:
            limit = self.max_detection_thresholds[-1]
            if max(len(item["labels"]) for item in preds) > limit:
                _warning_on_too_many_detections(limit)
        segm = "segm" in self.iou_type
        if segm:
            det_rle = _rle.encode([item["masks"] for item in preds])
            gt_rle = _rle.encode([item["masks"] for item in target])
        crowds = self._defaults_for(target, "iscrowd")
        areas = self._defaults_for(target, "area")
        det_n = [item["labels"].shape[0] if item["labels"].ndim else 1 for item in preds]
        gt_n = [item["labels"].shape[0] if item["labels"].ndim else 1 for item in target]
        columns = {
            "detection_labels": ([p["labels"] for p in preds], det_n),
            "detection_scores": ([p["scores"] for p in preds], det_n),
            "groundtruth_labels": ([t["labels"] for t in target], gt_n),
            "groundtruth_crowds": ([t["iscrowd"] if "iscrowd" in t else c for t, c in zip(target, crowds)], gt_n),
            "groundtruth_area": ([t["area"] if "area" in t else a for t, a in zip(target, areas)], gt_n),
        }
        if "bbox" in self.iou_type:
            columns["detection_box"] = ([_fix_empty_tensors(p["boxes"]) for p in preds], det_n)
            columns["groundtruth_box"] = ([_fix_empty_tensors(t["boxes"]) for t in target], gt_n)
        for name, (parts, sizes) in columns.items():
            flat = self._stack_images(parts, sizes, 4 if name in self._BOX_STATES else None)
            if flat is None:  # irregular images (mixed devices / dtypes / shapes): one list entry per image
                if name in self._BOX_STATES:
                    parts = self._convert_boxes(parts)
                getattr(self, name).extend(parts)
                continue
            if name in self._BOX_STATES and flat.numel():
                flat = box_convert(flat, in_fmt=self.box_format, out_fmt="xywh")
            self._append_chunk(name, flat, sizes)
        if segm:
            self.detection_mask.extend(det_rle)
            self.groundtruth_mask.extend(gt_rle)

    def _native_pack(self, preds: Any, target: Any) -> bool:
        """ROCm bbox batches: validation and packing of every image into the 7 flat states in one native call
        (``csrc/bindings/fastcall.cpp`` map_pack + ``csrc/detection/pack_images.hip``: one launch per 128 (image,
        state) segments, xyxy -> xywh fused into the copy).  False (nothing done) for anything else: the Python path
        below validates -- raising the reference's errors -- and packs."""
        if self.iou_type != ("bbox",) or not preds or not ops.native_available():
            return False
        box_mode = 1 if self.box_format == "xyxy" else 0
        got = ops.map_pack(preds, target, box_mode)
        if got is None:
            return False
        *flats, det_n, gt_n = got
        if self.warn_on_many_detections and max(det_n) > self.max_detection_thresholds[-1]:
            _warning_on_too_many_detections(self.max_detection_thresholds[-1])
        for name, flat in zip(self._NATIVE_ORDER, flats):
            if name in self._BOX_STATES and box_mode == 0 and self.box_format != "xywh" and flat.numel():
                flat = box_convert(flat, in_fmt=self.box_format, out_fmt="xywh")
            self._append_chunk(name, flat, det_n if name.startswith("detection") else gt_n)
        return True

    _NATIVE_ORDER = ("detection_box", "detection_scores", "detection_labels", "groundtruth_box", "groundtruth_labels",
                     "groundtruth_crowds", "groundtruth_area")

    @staticmethod
    def _stack_images(parts: List[Tensor], sizes: List[int], width: Optional[int]) -> Optional[Tensor]:
        """The images' tensors as one ``cat`` along dim 0 when they stack exactly (one device / dtype, ``[n_i]`` or
        ``[n_i, width]`` with ``n_i`` = the image's label count), else None."""
        first = parts[0]
        dev, dt = first.device, first.dtype
        if width is None:
            ok = all(p.ndim == 1 and p.device == dev and p.dtype == dt for p in parts)
        else:
            ok = all(p.ndim == 2 and p.shape[1] == width and p.device == dev and p.dtype == dt for p in parts)
        if not ok or any(p.shape[0] != n for p, n in zip(parts, sizes)):
            return None
        return torch.cat(parts) if len(parts) > 1 else first

    def _packed(self, name: str) -> Union[List[Tensor], "Packed"]:
        """List state ``name`` for the evaluator: flat (:class:`Packed`) when it stacks, else the list itself
        (memoised for the duration of one ``compute()``)."""
        memo = self.__dict__.get("_packed_memo")
        if memo is not None and name in memo:
            return memo[name]
        flat, sizes = self._packed_state(name)
        out = getattr(self, name) if flat is None else Packed(flat, sizes)
        if memo is not None:
            memo[name] = out
        return out

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
        memo = self.__dict__.get("_packed_memo")
        if memo is not None and "classes" in memo:  # (one unique + host read per compute(), not one per use)
            return memo["classes"]
        out = self._get_classes_uncached()
        if memo is not None:
            memo["classes"] = out
        return out

    def _get_classes_uncached(self) -> List[int]:
        return self._classes_both()[0]

    def _classes_both(self) -> Tuple[List[int], Optional[Tensor]]:
        """The sorted category ids present: the host list (the K axis) and the device tensor ``unique()`` produced
        (kept, instead of copying the list back: a host-to-device copy drains the stream)."""
        memo = self.__dict__.get("_packed_memo")
        if memo is not None and "classes_both" in memo:
            return memo["classes_both"]
        dev = self._state_device()
        parts = [cat_states(self._packed(n), dev).reshape(-1) for n in ("detection_labels", "groundtruth_labels")]
        # ROCm: one bitmap launch (labels in [0, 65536)); else torch.unique of the concatenation
        fast = ops.small_unique(parts[0], parts[1]) if parts[0].numel() + parts[1].numel() else None
        if fast is not None:
            out = fast
        else:
            labels = torch.cat([p.long() for p in parts])
            if labels.numel():
                u = labels.unique()
                out = (u.cpu().tolist(), u)
            else:
                out = ([], None)
        if memo is not None:
            memo["classes_both"] = out
        return out

    def _state_device(self) -> torch.device:
        for name in ("detection_labels", "groundtruth_labels"):
            st = self._packed(name)
            if isinstance(st, Packed):
                return st.flat.device
            if len(st):
                return st[0].device
        return self.device

    def _rle_states(self, dev: torch.device):
        """``(buffer, descriptors)`` of the detection and ground-truth mask packs (one descriptor row per mask)."""
        det = _rle.descriptors(self.detection_mask, image_sizes(self._packed("detection_labels")), dev)
        gt = _rle.descriptors(self.groundtruth_mask, image_sizes(self._packed("groundtruth_labels")), dev)
        return det, gt

    def _evaluate(self, i_type: str, micro: bool) -> Dict[str, Tensor]:
        dev = self._state_device()
        host_cls, dev_cls = self._classes_both()
        classes = dev_cls if dev_cls is not None and dev_cls.device == dev else \
            torch.tensor(host_cls, dtype=torch.long, device=dev)

        def relabel(xs):
            if not micro:
                return xs
            return xs.zeros_like() if isinstance(xs, Packed) else [torch.zeros_like(x) for x in xs]

        det_labels, gt_labels = self._packed("detection_labels"), self._packed("groundtruth_labels")
        n = len(det_labels)
        boxes_ok = i_type == "bbox"
        empty_box = torch.zeros(0, 4, device=dev)
        det_rle, gt_rle = self._rle_states(dev) if "segm" in self.iou_type else (None, None)
        gt_areas = self._packed("groundtruth_area")
        if len(self.iou_type) > 1:
            # with both iou types the reference keeps the ground-truth area of the mask for the bbox evaluation too
            a = cat_states(gt_areas, dev).reshape(-1)
            m = gt_rle[1][:, 2].to(dev, torch.float64)
            gt_areas = Packed(torch.where(a > 0, a.to(torch.float64), m), image_sizes(gt_labels))
        return coco_evaluate(
            det_boxes=self._packed("detection_box") if boxes_ok else [empty_box] * n,
            det_scores=self._packed("detection_scores"),
            det_labels=relabel(det_labels),
            gt_boxes=self._packed("groundtruth_box") if boxes_ok else [empty_box] * n,
            gt_labels=relabel(gt_labels),
            gt_crowds=self._packed("groundtruth_crowds"),
            gt_areas=gt_areas,
            iou_thresholds=self.iou_thresholds,
            rec_thresholds=self.rec_thresholds,
            max_dets=self.max_detection_thresholds,
            classes=classes,
            det_rle=None if boxes_ok else det_rle,
            gt_rle=None if boxes_ok else gt_rle,
        )

    def compute(self) -> dict:
        self.__dict__["_packed_memo"] = {}
        try:
            return self._compute()
        finally:
            self.__dict__.pop("_packed_memo", None)

    def _compute(self) -> dict:
        result: Dict[str, Tensor] = {}
        mdt = self.max_detection_thresholds
        for i_type in self.iou_type:
            prefix = "" if len(self.iou_type) == 1 else f"{i_type}_"
            ev = self._evaluate(i_type, micro=self.average == "micro")
            # pycocotools takes mAP at a hard-coded 100 detections (-1 without that threshold); faster-coco-eval
            # uses the largest threshold
            legacy = 100 if self.backend == "pycocotools" else None
            ev_cls = None
            if self.class_metrics:
                ev_cls = self._evaluate(i_type, micro=False) if self.average == "micro" else ev
            # the summary and the per-class numbers cross to the host in ONE transfer
            stats, mp, mr = summarize_all(ev, self.iou_thresholds, mdt, map_max_det=legacy, class_ev=ev_cls)
            stats = stats.to(torch.float32)
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
                map_pc, mar_pc = mp.to(torch.float32), mr.to(torch.float32)
            else:
                map_pc = torch.tensor([-1.0], dtype=torch.float32)
                mar_pc = torch.tensor([-1.0], dtype=torch.float32)
            result.update({f"{prefix}map_per_class": map_pc, f"{prefix}mar_{mdt[-1]}_per_class": mar_pc})
        result.update({"classes": torch.tensor(self._get_classes(), dtype=torch.int32)})
        return result

    def _ious(self, i_type: str) -> "IoUTable":
        """Per (image, class) IoU matrices -- detections in score order (max-dets truncated) x ground truths -- for every
        pair where the class occurs in the image.

        Batched: all images' detections and ground truths are keyed ``image * K + class``, ordered by (key, score)
        with one stable sort each, every (detection, ground truth) pair of a key is enumerated with prefix sums and all
        IoUs are evaluated in one pass (boxes elementwise, masks by one ``rle_iou`` launch), then copied to the host
        ONCE.  The reference gets the same dictionary from pycocotools' per-(image, class) Python loop; the previous
        version here synchronised twice per (image, class)."""
        classes = self._get_classes()
        n_img = len(self._packed("detection_labels"))
        if n_img == 0 or not classes:
            return IoUTable([], torch.zeros(0), np.zeros((0, 2), dtype=np.int64), np.zeros(0, dtype=np.int64))
        dev = self._state_device()
        cls_t = torch.tensor(classes, dtype=torch.long, device=dev)
        k = len(classes)
        max_det = self.max_detection_thresholds[-1]

        def flat(lst):
            sizes = torch.tensor(image_sizes(lst), device=dev)
            return cat_states(lst, dev), torch.repeat_interleave(torch.arange(len(lst), device=dev), sizes)

        d_lab, d_img = flat(self._packed("detection_labels"))
        g_lab, g_img = flat(self._packed("groundtruth_labels"))
        d_key = d_img * k + torch.searchsorted(cls_t, d_lab.long())
        g_key = g_img * k + torch.searchsorted(cls_t, g_lab.long())
        d_score = cat_states(self._packed("detection_scores"), dev)
        # detections: by key, then descending score (stable: ties keep their input order, as argsort(-s, stable))
        by_score = torch.argsort(-d_score, stable=True)
        d_order = by_score[torch.argsort(d_key[by_score], stable=True)]
        ks = d_key[d_order]
        nk = n_img * k
        d_cnt = torch.bincount(ks, minlength=nk)
        d_start = torch.cumsum(d_cnt, 0) - d_cnt
        rank = torch.arange(ks.numel(), device=dev) - d_start[ks]
        keep = rank < max_det
        d_order, ks = d_order[keep], ks[keep]
        d_cnt = torch.bincount(ks, minlength=nk)
        g_order = torch.argsort(g_key, stable=True)
        g_cnt = torch.bincount(g_key, minlength=nk)
        g_start = torch.cumsum(g_cnt, 0) - g_cnt
        present = torch.nonzero((d_cnt > 0) | (g_cnt > 0)).flatten()
        # pairs: detection i (sorted) x every ground truth of its key
        per_det = g_cnt[ks]
        pair_det = torch.repeat_interleave(torch.arange(ks.numel(), device=dev), per_det)
        pair_start = torch.cumsum(per_det, 0) - per_det
        within = torch.arange(pair_det.numel(), device=dev) - pair_start[pair_det]
        pd = d_order[pair_det]
        pg = g_order[g_start[ks[pair_det]] + within]
        if i_type == "bbox":
            db = cat_states(self._packed("detection_box"), dev, (4,)).double()
            gb = cat_states(self._packed("groundtruth_box"), dev, (4,)).double()
            crowd = cat_states(self._packed("groundtruth_crowds"), dev).bool()
            d, g = db[pd], gb[pg]
            x1, y1 = torch.maximum(d[:, 0], g[:, 0]), torch.maximum(d[:, 1], g[:, 1])
            x2 = torch.minimum(d[:, 0] + d[:, 2], g[:, 0] + g[:, 2])
            y2 = torch.minimum(d[:, 1] + d[:, 3], g[:, 1] + g[:, 3])
            w, h = x2 - x1, y2 - y1
            inter = torch.where((w > 0) & (h > 0), w * h, torch.zeros_like(w))
            da = d[:, 2] * d[:, 3]
            union = torch.where(crowd[pg], da, da + g[:, 2] * g[:, 3] - inter)
            vals = torch.where(inter > 0, inter / union, torch.zeros_like(inter)).float()
        else:
            (dbuf, ddesc), (gbuf, gdesc) = self._rle_states(dev)
            g_crowd = cat_states(self._packed("groundtruth_crowds"), gdesc.device).reshape(-1).clamp(0, 1)
            g_crowd = g_crowd.to(torch.uint8) if g_crowd.numel() else torch.zeros(0, dtype=torch.uint8,
                                                                                device=gdesc.device)
            vals = ops.rle_iou(dbuf, ddesc, gbuf, gdesc, pd.to(ddesc.device).contiguous(),
                               pg.to(ddesc.device).contiguous(), g_crowd).float()
        # ONE host transfer: the values and the per-key shapes (pairs of a key are contiguous, row-major)
        shapes = torch.stack([d_cnt[present], g_cnt[present]], 1)
        pair_cnt = d_cnt * g_cnt
        offs = (torch.cumsum(pair_cnt, 0) - pair_cnt)[present]
        host = torch.cat([present.double(), shapes.reshape(-1).double(), offs.double(), vals.double()]).cpu()
        npres = present.numel()
        pres = host[:npres].long().numpy()
        img, cls = pres // k, np.asarray(classes, dtype=np.int64)[pres % k]
        shp = host[npres: 3 * npres].long().reshape(-1, 2).numpy()
        off = host[3 * npres: 4 * npres].long().numpy()
        return IoUTable((img, cls), host[4 * npres:].float(), shp, off)

    # ---------------------------------------------------------------------------------------- COCO interop
    def tm_to_coco(self, name: str = "tm_map_input") -> None:
        """Write the accumulated annotations as COCO json files ``{name}_preds.json`` / ``{name}_target.json``
        (boxes as xywh ``bbox``; masks as compressed-RLE ``segmentation`` built from the stored runs)."""
        bbox, segm = "bbox" in self.iou_type, "segm" in self.iou_type

        def fmt(labels, boxes, masks, scores=None, crowds=None, areas=None):
            images, anns, aid = [], [], 1
            for img, lab in enumerate(labels):
                rles = _rle.pack_to_coco(masks[img]) if segm else []
                if segm and not rles and not bbox:
                    continue
                images.append({"id": img})
                if rles:
                    images[-1]["height"], images[-1]["width"] = rles[0]["size"]
                b = boxes[img].reshape(-1, 4).cpu().tolist() if bbox else []
                for k, label in enumerate(lab.cpu().tolist()):
                    if areas is not None and float(areas[img][k]) > 0:
                        area = float(areas[img][k])
                    else:
                        area = float(self._rle_area(masks[img], k)) if segm else b[k][2] * b[k][3]
                    ann = {"id": aid, "image_id": img, "area": area, "category_id": int(label),
                           "iscrowd": int(crowds[img][k]) if crowds is not None else 0}
                    if bbox:
                        ann["bbox"] = b[k]
                    if rles:
                        ann["segmentation"] = rles[k]
                    if scores is not None:
                        ann["score"] = float(scores[img][k])
                    anns.append(ann)
                    aid += 1
            cats = [{"id": i, "name": str(i)} for i in self._get_classes()]
            return {"images": images, "annotations": anns, "categories": cats}

        target = fmt(self.groundtruth_labels, self.groundtruth_box, self.groundtruth_mask,
                     crowds=self.groundtruth_crowds, areas=self.groundtruth_area)
        preds = fmt(self.detection_labels, self.detection_box, self.detection_mask, scores=self.detection_scores)
        with open(f"{name}_preds.json", "w") as f:
            f.write(json.dumps(preds["annotations"], indent=4))
        with open(f"{name}_target.json", "w") as f:
            f.write(json.dumps(target, indent=4))

    @staticmethod
    def _rle_area(pack: Tensor, k: int) -> int:
        return int(pack[3 + k].item())

    @staticmethod
    def coco_to_tm(
        coco_preds: str,
        coco_target: str,
        iou_type: Union[Literal["bbox", "segm"], List[str]] = "bbox",
        backend: Literal["pycocotools", "faster_coco_eval"] = "pycocotools",
    ) -> Tuple[List[Dict[str, Tensor]], List[Dict[str, Tensor]]]:
        """Read COCO json (target dataset + prediction list) into the ``update`` input format.

        ``segm`` annotations may be polygons, uncompressed RLE or compressed RLE; masks are rasterised at the image's
        ``height`` x ``width`` (``images`` entries of the target file) as ``uint8 [n, H, W]``, like the reference's
        ``annToMask`` (``S/detection/mean_ap.py:694-747``).
        """
        iou_type = _validate_iou_type_arg(iou_type)
        bbox, segm = "bbox" in iou_type, "segm" in iou_type
        with open(coco_target) as f:
            gt = json.load(f)
        with open(coco_preds) as f:
            dt = json.load(f)
        # images in order of their first ground-truth annotation (images without ground truth are not evaluated)
        order = list(dict.fromkeys(ann["image_id"] for ann in gt["annotations"]))
        sizes = {img["id"]: (img.get("height"), img.get("width")) for img in gt.get("images", [])}

        def mask_of(ann):
            h, w = sizes.get(ann["image_id"], (None, None))
            seg = ann["segmentation"]
            if (h is None or w is None) and isinstance(seg, dict):
                h, w = seg["size"]
            if h is None or w is None:
                raise ValueError(f"coco_to_tm: image {ann['image_id']} has no height / width for its segmentation")
            return _rle.segmentation_to_mask(seg, int(h), int(w))

        def new_entry(image_id, with_scores):
            e = {"boxes": [], "labels": [], "masks": []}
            e.update({"scores": []} if with_scores else {"iscrowd": [], "area": []})
            return e

        target = {i: new_entry(i, False) for i in order}
        for ann in gt["annotations"]:
            t = target[ann["image_id"]]
            if bbox:
                t["boxes"].append(ann["bbox"])
            if segm:
                t["masks"].append(mask_of(ann))
            t["labels"].append(ann["category_id"])
            t["iscrowd"].append(ann.get("iscrowd", 0))
            t["area"].append(ann.get("area", 0.0))
        preds = {i: new_entry(i, True) for i in order}
        for ann in dt:
            p = preds.setdefault(ann["image_id"], new_entry(ann["image_id"], True))
            if bbox:
                p["boxes"].append(ann["bbox"])
            if segm:
                p["masks"].append(mask_of(ann))
            p["labels"].append(ann["category_id"])
            p["scores"].append(ann["score"])

        def masks_tensor(lst, image_id):
            if lst:
                return torch.from_numpy(np.stack(lst)).to(torch.uint8)
            h, w = sizes.get(image_id, (0, 0))
            return torch.zeros(0, int(h or 0), int(w or 0), dtype=torch.uint8)

        bp, bt = [], []
        for key in order:
            p, t = preds[key], target[key]
            ep = {"scores": torch.tensor(p["scores"], dtype=torch.float32),
                  "labels": torch.tensor(p["labels"], dtype=torch.int32)}
            et = {"labels": torch.tensor(t["labels"], dtype=torch.int32),
                  "iscrowd": torch.tensor(t["iscrowd"], dtype=torch.int32),
                  "area": torch.tensor(t["area"], dtype=torch.float32)}
            if bbox:
                ep["boxes"] = torch.tensor(p["boxes"], dtype=torch.float32).reshape(-1, 4)
                et["boxes"] = torch.tensor(t["boxes"], dtype=torch.float32).reshape(-1, 4)
            if segm:
                ep["masks"] = masks_tensor(p["masks"], key)
                et["masks"] = masks_tensor(t["masks"], key)
            bp.append(ep)
            bt.append(et)
        return bp, bt


class IoUTable(Mapping):
    """``{(image, class): IoU matrix}`` backed by ONE flat host tensor; each matrix is a view made on access (the
    extended-summary ``ious`` of tens of thousands of (image, class) pairs costs no per-entry tensor up front).  The keys
    are two integer arrays; the tuple keys and the lookup index are only built when the mapping is first iterated /
    indexed, so ``compute()`` itself does no per-pair Python work."""

    def __init__(self, keys: Any, values: Tensor, shapes: Any, offsets: Any) -> None:
        if isinstance(keys, tuple) and len(keys) == 2 and isinstance(keys[0], np.ndarray):
            self._img, self._cls = keys
        else:  # a list of (image, class) tuples
            arr = np.asarray(keys, dtype=np.int64).reshape(-1, 2)
            self._img, self._cls = arr[:, 0], arr[:, 1]
        self._values = values
        self._shapes = np.asarray(shapes, dtype=np.int64).reshape(-1, 2)
        self._offsets = np.asarray(offsets, dtype=np.int64).reshape(-1)
        self._index: Optional[Dict[Tuple[int, int], int]] = None
        self._key_list: Optional[List[Tuple[int, int]]] = None

    def _keys(self) -> List[Tuple[int, int]]:
        if self._key_list is None:
            self._key_list = list(zip(self._img.tolist(), self._cls.tolist()))
        return self._key_list

    def __getitem__(self, key: Tuple[int, int]) -> Tensor:
        if self._index is None:
            self._index = {kk: i for i, kk in enumerate(self._keys())}
        i = self._index[key]
        n, m = int(self._shapes[i, 0]), int(self._shapes[i, 1])
        o = int(self._offsets[i])
        if n * m == 1:  # compute() results go through _squeeze_if_scalar: a 1 x 1 matrix comes out 0-d, as there
            return self._values[o]
        return self._values[o: o + n * m].view(n, m)

    def __iter__(self):
        return iter(self._keys())

    def __len__(self) -> int:
        return int(self._img.shape[0])

    def __repr__(self) -> str:
        return f"IoUTable({len(self)} (image, class) pairs)"

    _tm_flat_mapping = True

    def apply_flat(self, fn: Any) -> Any:
        """``fn`` applied to every matrix, evaluated once on the flat storage when that is equivalent (a device /
        dtype move keeps the element count); otherwise per matrix into a plain dict."""
        out = fn(self._values)
        if isinstance(out, Tensor) and out.numel() == self._values.numel() and out.dim() == 1:
            return IoUTable((self._img, self._cls), out, self._shapes, self._offsets)
        return {k: fn(self[k]) for k in self._keys()}


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
