"""IoU / GIoU / DIoU / CIoU module metrics on the ragged one-launch path (``ops.box_pairwise_ragged`` +
``ops.iou_class_reduce``) against the reference algorithm written out per image and per class
(S/detection/iou.py:180-221, torchvision box-op formulas), for every box format, threshold / label / class option,
images without detections or ground truths, and the state layout (per-image ``[n_i, m_i]`` matrices)."""
import math

import pytest
import torch

from torchmetrics_amd.detection import (
    CompleteIntersectionOverUnion,
    DistanceIntersectionOverUnion,
    GeneralizedIntersectionOverUnion,
    IntersectionOverUnion,
)


def _pair(a, b, kind):
    a, b = a.double()[:, None], b.double()[None]
    area_a = (a[..., 2] - a[..., 0]) * (a[..., 3] - a[..., 1])
    area_b = (b[..., 2] - b[..., 0]) * (b[..., 3] - b[..., 1])
    iw = (torch.minimum(a[..., 2], b[..., 2]) - torch.maximum(a[..., 0], b[..., 0])).clamp(min=0)
    ih = (torch.minimum(a[..., 3], b[..., 3]) - torch.maximum(a[..., 1], b[..., 1])).clamp(min=0)
    inter = iw * ih
    union = area_a + area_b - inter
    iou = inter / union
    if kind == "iou":
        return iou
    cw = torch.maximum(a[..., 2], b[..., 2]) - torch.minimum(a[..., 0], b[..., 0])
    ch = torch.maximum(a[..., 3], b[..., 3]) - torch.minimum(a[..., 1], b[..., 1])
    if kind == "giou":
        return iou - (cw * ch - union) / (cw * ch)
    diag = cw**2 + ch**2 + 1e-7
    dx = (a[..., 0] + a[..., 2]) / 2 - (b[..., 0] + b[..., 2]) / 2
    dy = (a[..., 1] + a[..., 3]) / 2 - (b[..., 1] + b[..., 3]) / 2
    diou = iou - (dx**2 + dy**2) / diag
    if kind == "diou":
        return diou
    wa, ha, wb, hb = a[..., 2] - a[..., 0], a[..., 3] - a[..., 1], b[..., 2] - b[..., 0], b[..., 3] - b[..., 1]
    v = (4 / math.pi**2) * (torch.atan(wb / hb) - torch.atan(wa / ha)) ** 2
    alpha = v / (1 - iou + v + 1e-7)
    return diou - alpha * v


def _to_xyxy(b, fmt):
    if fmt == "xywh":
        return torch.stack([b[:, 0], b[:, 1], b[:, 0] + b[:, 2], b[:, 1] + b[:, 3]], -1)
    if fmt == "cxcywh":
        return torch.stack([b[:, 0] - b[:, 2] / 2, b[:, 1] - b[:, 3] / 2, b[:, 0] + b[:, 2] / 2,
                            b[:, 1] + b[:, 3] / 2], -1)
    return b


def _reference(preds, target, kind, invalid, fmt, thr, respect, class_metrics):
    mats, labs = [], []
    for p, t in zip(preds, target):
        mat = _pair(_to_xyxy(p["boxes"], fmt), _to_xyxy(t["boxes"], fmt), kind)
        if thr is not None:
            mat[mat < thr] = invalid
        if respect:
            mat[~(p["labels"][:, None] == t["labels"][None])] = invalid
        mats.append(mat)
        labs.append(t["labels"])
    out = {kind: torch.cat([mt[mt != invalid] for mt in mats]).mean()}
    if class_metrics:
        for cl in torch.cat(labs).unique().tolist():
            s, c = 0.0, 0
            for mt, lab in zip(mats, labs):
                sc = mt[:, lab == cl]
                s += float(sc[sc != invalid].sum())
                c += int((sc != invalid).sum())
            out[f"{kind}/cl_{cl}"] = torch.tensor(s / c if c else float("nan"))
    return out


def _data(n_img=12, seed=0, fmt="xyxy"):
    g = torch.Generator().manual_seed(seed)
    preds, target = [], []
    for i in range(n_img):
        nd, ng = (0 if i == 3 else int(torch.randint(1, 9, (1,), generator=g))), (0 if i == 5 else
                                                                                  int(torch.randint(1, 7, (1,), generator=g)))

        def boxes(k):
            xy = torch.rand(k, 2, generator=g) * 80
            wh = torch.rand(k, 2, generator=g) * 40 + 2
            b = torch.cat([xy, xy + wh], -1)
            if fmt == "xywh":
                b = torch.cat([xy, wh], -1)
            elif fmt == "cxcywh":
                b = torch.cat([xy + wh / 2, wh], -1)
            return b

        preds.append({"boxes": boxes(nd), "labels": torch.randint(0, 3, (nd,), generator=g)})
        target.append({"boxes": boxes(ng), "labels": torch.randint(0, 3, (ng,), generator=g)})
    return preds, target


CLASSES = [(IntersectionOverUnion, "iou", -1.0), (GeneralizedIntersectionOverUnion, "giou", -1.0),
           (DistanceIntersectionOverUnion, "diou", -1.0), (CompleteIntersectionOverUnion, "ciou", -2.0)]


@pytest.mark.parametrize(("cls", "kind", "invalid"), CLASSES)
@pytest.mark.parametrize("fmt", ["xyxy", "xywh", "cxcywh"])
@pytest.mark.parametrize(("thr", "respect", "class_metrics"), [(None, True, True), (0.2, False, True),
                                                               (None, False, False), (0.1, True, False)])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_iou_family_matches_reference_algorithm(cls, kind, invalid, fmt, thr, respect, class_metrics, device):
    preds, target = _data(fmt=fmt)
    m = cls(box_format=fmt, iou_threshold=thr, respect_labels=respect, class_metrics=class_metrics).to(device)
    dev = lambda xs: [{k: v.to(device) for k, v in x.items()} for x in xs]  # noqa: E731
    m.update(dev(preds[:7]), dev(target[:7]))
    m.update(dev(preds[7:]), dev(target[7:]))
    assert len(m.iou_matrix) == 12 and m.iou_matrix[4].shape == (preds[4]["boxes"].shape[0], target[4]["boxes"].shape[0])
    out = m.compute()
    ref = _reference(preds, target, kind, invalid, fmt, thr, respect, class_metrics)
    assert set(out) == set(ref)
    for k in ref:
        torch.testing.assert_close(out[k].cpu().double(), ref[k].double(), atol=1e-5, rtol=1e-5, equal_nan=True)
