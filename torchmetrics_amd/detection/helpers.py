"""Detection input validation and box utilities (behaviour of reference ``S/detection/helpers.py``)."""
from typing import Any, Dict, Literal, Sequence, Tuple, Union

import torch
from torch import Tensor


def _input_validator(
    preds: Sequence[Dict[str, Tensor]],
    targets: Sequence[Dict[str, Tensor]],
    iou_type: Union[Literal["bbox", "segm"], Tuple[Literal["bbox", "segm"]]] = "bbox",
    ignore_score: bool = False,
) -> None:
    """Check the list-of-dicts detection inputs (keys, types, per-sample lengths).

    One pass over the images for valid inputs (a detection batch of 512 images is validated in a fraction of the
    time the check-by-check passes take); anything it does not accept goes through the full sequence of checks,
    which raises the reference's error for the first failing check."""
    if _inputs_ok(preds, targets, iou_type, ignore_score):
        return
    _input_validator_full(preds, targets, iou_type, ignore_score)


def _inputs_ok(preds: Any, targets: Any, iou_type: Any, ignore_score: bool) -> bool:
    if not isinstance(preds, (list, tuple)) or not isinstance(targets, (list, tuple)) or len(preds) != len(targets):
        return False
    if isinstance(iou_type, str):
        iou_type = (iou_type,)
    if iou_type == ("bbox",):
        key = "boxes"
    elif iou_type == ("segm",):
        key = "masks"
    else:
        return False
    T = Tensor
    try:
        for t in targets:
            b, lab = t[key], t["labels"]
            if type(b) is not T and not isinstance(b, T) or type(lab) is not T and not isinstance(lab, T):
                return False
            if b.size(0) != lab.size(0):
                return False
        for p in preds:
            b, lab = p[key], p["labels"]
            if type(b) is not T and not isinstance(b, T) or type(lab) is not T and not isinstance(lab, T):
                return False
            if ignore_score:
                continue
            sc = p["scores"]
            if type(sc) is not T and not isinstance(sc, T):
                return False
            if not (b.size(0) == lab.size(0) == sc.size(0)):
                return False
    except (KeyError, TypeError, IndexError, RuntimeError):
        return False
    return True


def _input_validator_full(
    preds: Sequence[Dict[str, Tensor]],
    targets: Sequence[Dict[str, Tensor]],
    iou_type: Union[Literal["bbox", "segm"], Tuple[Literal["bbox", "segm"]]] = "bbox",
    ignore_score: bool = False,
) -> None:
    if isinstance(iou_type, str):
        iou_type = (iou_type,)
    name_map = {"bbox": "boxes", "segm": "masks"}
    if any(tp not in name_map for tp in iou_type):
        raise Exception(f"IOU type {iou_type} is not supported")
    keys = [name_map[tp] for tp in iou_type]
    if not isinstance(preds, Sequence):
        raise ValueError(f"Expected argument `preds` to be of type Sequence, but got {preds}")
    if not isinstance(targets, Sequence):
        raise ValueError(f"Expected argument `target` to be of type Sequence, but got {targets}")
    if len(preds) != len(targets):
        raise ValueError(
            f"Expected argument `preds` and `target` to have the same length, but got {len(preds)} and {len(targets)}"
        )
    for k in [*keys, "labels"] + ([] if ignore_score else ["scores"]):
        if any(k not in p for p in preds):
            raise ValueError(f"Expected all dicts in `preds` to contain the `{k}` key")
    for k in [*keys, "labels"]:
        if any(k not in p for p in targets):
            raise ValueError(f"Expected all dicts in `target` to contain the `{k}` key")
    for k in keys:
        if not all(isinstance(p[k], Tensor) for p in preds):
            raise ValueError(f"Expected all {k} in `preds` to be of type Tensor")
    if not ignore_score and not all(isinstance(p["scores"], Tensor) for p in preds):
        raise ValueError("Expected all scores in `preds` to be of type Tensor")
    if not all(isinstance(p["labels"], Tensor) for p in preds):
        raise ValueError("Expected all labels in `preds` to be of type Tensor")
    for k in keys:
        if not all(isinstance(t[k], Tensor) for t in targets):
            raise ValueError(f"Expected all {k} in `target` to be of type Tensor")
    if not all(isinstance(t["labels"], Tensor) for t in targets):
        raise ValueError("Expected all labels in `target` to be of type Tensor")
    for i, item in enumerate(targets):
        for k in keys:
            if item[k].size(0) != item["labels"].size(0):
                raise ValueError(
                    f"Input '{k}' and labels of sample {i} in targets have a"
                    f" different length (expected {item[k].size(0)} labels, got {item['labels'].size(0)})"
                )
    if ignore_score:
        return
    for i, item in enumerate(preds):
        for k in keys:
            if not (item[k].size(0) == item["labels"].size(0) == item["scores"].size(0)):
                raise ValueError(
                    f"Input '{k}', labels and scores of sample {i} in predictions have a"
                    f" different length (expected {item[k].size(0)} labels and scores,"
                    f" got {item['labels'].size(0)} labels and {item['scores'].size(0)})"
                )


def _fix_empty_tensors(boxes: Tensor) -> Tensor:
    """Empty 1-D box tensors become ``[0, 4]`` ... well, ``[1, 0]`` as the reference (kept for state parity)."""
    if boxes.numel() == 0 and boxes.ndim == 1:
        return boxes.unsqueeze(0)
    return boxes


def _validate_iou_type_arg(iou_type: Union[Literal["bbox", "segm"], Tuple[str]] = "bbox") -> Tuple[str]:
    allowed = ("segm", "bbox")
    if isinstance(iou_type, str):
        iou_type = (iou_type,)
    if any(tp not in allowed for tp in iou_type):
        raise ValueError(f"Expected argument `iou_type` to be one of {allowed} or a list of, but got {iou_type}")
    return iou_type


def box_convert(boxes: Tensor, in_fmt: str, out_fmt: str) -> Tensor:
    """Convert ``[N, 4]`` boxes between ``xyxy``, ``xywh`` and ``cxcywh`` (torchvision ``box_convert`` semantics)."""
    allowed = ("xyxy", "xywh", "cxcywh")
    if in_fmt not in allowed or out_fmt not in allowed:
        raise ValueError(f"Unsupported Bounding Box Conversions for given in_fmt {in_fmt} and out_fmt {out_fmt}")
    if in_fmt == out_fmt:
        return boxes.clone()
    a, b, c, d = boxes.unbind(-1)
    if in_fmt == "xywh":
        x1, y1, x2, y2 = a, b, a + c, b + d
    elif in_fmt == "cxcywh":
        x1, y1, x2, y2 = a - 0.5 * c, b - 0.5 * d, a + 0.5 * c, b + 0.5 * d
    else:
        x1, y1, x2, y2 = a, b, c, d
    if out_fmt == "xyxy":
        return torch.stack([x1, y1, x2, y2], -1)
    if out_fmt == "xywh":
        return torch.stack([x1, y1, x2 - x1, y2 - y1], -1)
    return torch.stack([(x1 + x2) / 2, (y1 + y2) / 2, x2 - x1, y2 - y1], -1)
