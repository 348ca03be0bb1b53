"""Detection: IoU family kernels, MeanAveragePrecision vs a plain-Python COCO oracle and published fixture values."""
import numpy as np
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.detection import MeanAveragePrecision
from tests._coco_oracle import coco_eval, summarize
from tests.helpers import assert_close, run_ddp

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
IOU_THRS = torch.linspace(0.5, 0.95, 10).tolist()
REC_THRS = torch.linspace(0.0, 1.0, 101).tolist()


def _random_coco(seed, n_img=12, n_cls=4, max_gt=8, max_det=15, crowd=True):
    g = torch.Generator().manual_seed(seed)
    preds, target = [], []
    for _ in range(n_img):
        ng = int(torch.randint(0, max_gt + 1, (1,), generator=g))
        nd = int(torch.randint(0, max_det + 1, (1,), generator=g))
        gxy = torch.rand(ng, 2, generator=g) * 200
        gwh = torch.rand(ng, 2, generator=g) * 120 + 4
        gb = torch.cat([gxy, gxy + gwh], 1)
        gl = torch.randint(0, n_cls, (ng,), generator=g)
        # detections: jittered copies of ground truths plus clutter
        src = torch.randint(0, max(ng, 1), (nd,), generator=g)
        jitter = torch.randn(nd, 4, generator=g) * 6
        db = gb[src] + jitter if ng else torch.rand(nd, 4, generator=g) * 200
        db = torch.cat([torch.minimum(db[:, :2], db[:, 2:]), torch.maximum(db[:, :2], db[:, 2:]) + 1], 1)
        dl = gl[src] if ng else torch.randint(0, n_cls, (nd,), generator=g)
        flip = torch.rand(nd, generator=g) < 0.2
        dl = torch.where(flip, torch.randint(0, n_cls, (nd,), generator=g), dl)
        scores = (torch.rand(nd, generator=g) * 10).round() / 10  # ties
        t = {"boxes": gb, "labels": gl}
        if crowd:
            t["iscrowd"] = (torch.rand(ng, generator=g) < 0.15).long()
        preds.append({"boxes": db, "scores": scores, "labels": dl})
        target.append(t)
    return preds, target


def _oracle(preds, target, max_dets=(1, 10, 100)):
    def xywh(b):
        return [[x1, y1, x2 - x1, y2 - y1] for x1, y1, x2, y2 in b.tolist()]

    cats = sorted(set(torch.cat([p["labels"] for p in preds] + [t["labels"] for t in target]).tolist()))
    dets = [[(bb, s, c) for bb, s, c in zip(xywh(p["boxes"]), p["scores"].tolist(), p["labels"].tolist())]
            for p in preds]
    gts = []
    for t in target:
        bb = xywh(t["boxes"])
        crowd = t.get("iscrowd", torch.zeros_like(t["labels"])).tolist()
        gts.append([(b, c, cr, b[2] * b[3]) for b, c, cr in zip(bb, t["labels"].tolist(), crowd)])
    prec, rec = coco_eval(dets, gts, cats, IOU_THRS, REC_THRS, list(max_dets))
    return summarize(prec, rec, IOU_THRS, list(max_dets)), prec, rec


def _to(items, device):
    return [{k: v.to(device) for k, v in it.items()} for it in items]


# ---------------------------------------------------------------------------------------------------- box ops
@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("op", [ops.BOX_IOU, ops.BOX_GIOU, ops.BOX_DIOU, ops.BOX_CIOU])
def test_box_pairwise_matches_formula(device, op):
    g = torch.Generator().manual_seed(op)
    a = torch.rand(37, 2, generator=g) * 50
    a = torch.cat([a, a + torch.rand(37, 2, generator=g) * 30 + 1], 1)
    b = torch.rand(23, 2, generator=g) * 50
    b = torch.cat([b, b + torch.rand(23, 2, generator=g) * 30 + 1], 1)
    ref = ops._cpu.box_pairwise(a.double(), b.double(), op, False)
    out = ops.box_pairwise(a.to(device), b.to(device), op)
    assert_close(out, ref, atol=1e-5)
    aligned = ops.box_pairwise(a[:23].to(device), b.to(device), op, aligned=True)
    assert_close(aligned, ref[:23].diagonal(), atol=1e-5)
    # torchvision-style reference for plain IoU
    if op == ops.BOX_IOU:
        area = lambda x: (x[:, 2] - x[:, 0]) * (x[:, 3] - x[:, 1])  # noqa: E731
        lt = torch.max(a[:, None, :2], b[None, :, :2])
        rb = torch.min(a[:, None, 2:], b[None, :, 2:])
        inter = (rb - lt).clamp(min=0).prod(2)
        assert_close(out, inter / (area(a)[:, None] + area(b)[None] - inter), atol=1e-5)


# ------------------------------------------------------------------------------------------------------- mAP
@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_map_vs_python_coco_oracle(device, seed):
    preds, target = _random_coco(seed)
    m = MeanAveragePrecision(class_metrics=True, extended_summary=True).to(device)
    m.update(_to(preds[:6], device), _to(target[:6], device))
    m.update(_to(preds[6:], device), _to(target[6:], device))
    res = m.compute()
    stats, prec, rec = _oracle(preds, target)
    names = ["map", "map_50", "map_75", "map_small", "map_medium", "map_large", "mar_1", "mar_10", "mar_100",
             "mar_small", "mar_medium", "mar_large"]
    for name, v in zip(names, stats):
        assert_close(res[name], v, atol=1e-6)
    assert_close(res["precision"], prec, atol=1e-6)
    assert_close(res["recall"], rec, atol=1e-6)
    # per-class: mean over (iou, recall) of the class slice at area=all, maxdet=100
    for k in range(prec.shape[2]):
        s = prec[:, :, k, 0, -1]
        exp = s[s > -1].mean() if (s > -1).any() else -1
        assert_close(res["map_per_class"][k], exp, atol=1e-6)


@pytest.mark.parametrize("device", DEVICES)
def test_map_max_dets_and_micro(device):
    preds, target = _random_coco(5, n_img=6, max_det=30)
    m = MeanAveragePrecision(max_detection_thresholds=[2, 5, 20], backend="faster_coco_eval").to(device)
    m.update(_to(preds, device), _to(target, device))
    res = m.compute()
    stats, _, _ = _oracle(preds, target, max_dets=(2, 5, 20))
    for name, v in zip(["map", "mar_2", "mar_5", "mar_20"], [stats[0], stats[6], stats[7], stats[8]]):
        assert_close(res[name], v, atol=1e-6)
    # pycocotools' summarize takes mAP at a hard-coded 100 detections: -1 without that threshold, the rest unchanged
    legacy = MeanAveragePrecision(max_detection_thresholds=[2, 5, 20]).to(device)
    legacy.update(_to(preds, device), _to(target, device))
    rl = legacy.compute()
    assert float(rl["map"]) == -1.0
    for name in ("map_50", "map_75", "mar_2", "mar_5", "mar_20"):
        assert_close(rl[name], res[name], atol=1e-7)
    mm = MeanAveragePrecision(average="micro").to(device)
    mm.update(_to(preds, device), _to(target, device))
    zero = [{**p, "labels": torch.zeros_like(p["labels"])} for p in preds]
    zt = [{**t, "labels": torch.zeros_like(t["labels"])} for t in target]
    stats_micro, _, _ = _oracle(zero, zt)
    assert_close(mm.compute()["map"], stats_micro[0], atol=1e-6)


# reference test fixture (``T/detection/test_map.py`` ``_inputs``: COCO val2014 image ids 42, 73, 74, 987).  The
# reference pins it against pycocotools at test time; pycocotools is not installable here, so the expected values
# come from the plain-Python COCO oracle (``tests/_coco_oracle.py``) -- parity with pycocotools itself is unpinned.
_FIXTURE_PREDS = [
    {"boxes": [[258.15, 41.29, 606.41, 285.07]], "scores": [0.236], "labels": [4]},
    {"boxes": [[61.00, 22.75, 565.00, 632.42], [12.66, 3.32, 281.26, 275.23]], "scores": [0.318, 0.726],
     "labels": [3, 2]},
    {"boxes": [[87.87, 276.25, 384.29, 379.43], [0.00, 3.66, 142.15, 316.06], [296.55, 93.96, 314.97, 152.79],
               [328.94, 97.05, 342.49, 122.98], [356.62, 95.47, 372.33, 147.55], [464.08, 105.09, 495.74, 146.99],
               [276.11, 103.84, 291.44, 150.72]],
     "scores": [0.546, 0.3, 0.407, 0.611, 0.335, 0.805, 0.953], "labels": [4, 1, 0, 0, 0, 0, 0]},
    {"boxes": [[72.92, 45.96, 91.23, 80.57], [45.17, 45.34, 66.28, 79.83], [82.28, 47.04, 99.66, 78.50],
               [59.96, 46.17, 80.35, 80.48], [75.29, 23.01, 91.85, 50.85], [71.14, 1.10, 96.96, 28.33],
               [61.34, 55.23, 77.14, 79.57], [41.17, 45.78, 60.99, 78.48], [56.18, 44.80, 64.42, 56.25]],
     "scores": [0.532, 0.204, 0.782, 0.202, 0.883, 0.271, 0.561, 0.204, 0.349], "labels": [49] * 9},
]
_FIXTURE_TARGET = [
    {"boxes": [[214.1500, 41.2900, 562.4100, 285.0700]], "labels": [4]},
    {"boxes": [[13.00, 22.75, 548.98, 632.42], [1.66, 3.32, 270.26, 275.23]], "labels": [2, 2]},
    {"boxes": [[61.87, 276.25, 358.29, 379.43], [2.75, 3.66, 162.15, 316.06], [295.55, 93.96, 313.97, 152.79],
               [326.94, 97.05, 340.49, 122.98], [356.62, 95.47, 372.33, 147.55], [462.08, 105.09, 493.74, 146.99],
               [277.11, 103.84, 292.44, 150.72]], "labels": [4, 1, 0, 0, 0, 0, 0]},
    {"boxes": [[72.92, 45.96, 91.23, 80.57], [50.17, 45.34, 71.28, 79.83], [81.28, 47.04, 98.66, 78.50],
               [63.96, 46.17, 84.35, 80.48], [75.29, 23.01, 91.85, 50.85], [56.39, 21.65, 75.66, 45.54],
               [73.14, 1.10, 98.96, 28.33], [62.34, 55.23, 78.14, 79.57], [44.17, 45.78, 63.99, 78.48],
               [58.18, 44.80, 66.42, 56.25]], "labels": [49] * 10},
]


@pytest.mark.parametrize("device", DEVICES)
def test_map_published_fixture(device):
    def conv(items, with_scores):
        out = []
        for it in items:
            d = {"boxes": torch.tensor(it["boxes"]), "labels": torch.tensor(it["labels"], dtype=torch.int32)}
            if with_scores:
                d["scores"] = torch.tensor(it["scores"])
            out.append(d)
        return out

    preds, target = conv(_FIXTURE_PREDS, True), conv(_FIXTURE_TARGET, False)
    m = MeanAveragePrecision(class_metrics=True).to(device)
    m.update(_to(preds, device), _to(target, device))
    res = m.compute()
    stats, _, _ = _oracle(preds, target)
    names = ["map", "map_50", "map_75", "map_small", "map_medium", "map_large", "mar_1", "mar_10", "mar_100",
             "mar_small", "mar_medium", "mar_large"]
    for name, v in zip(names, stats):
        assert_close(res[name], v, atol=1e-6)


def test_map_segm_matches_box_equivalent_masks():
    # masks that are exactly the (integer) boxes give the same IoU as COCO's box IoU
    g = torch.Generator().manual_seed(7)
    preds, target = [], []
    for _ in range(4):
        gt = torch.randint(0, 40, (5, 2), generator=g)
        gt = torch.cat([gt, gt + torch.randint(4, 20, (5, 2), generator=g)], 1)
        dt = (gt + torch.randint(-3, 4, (5, 4), generator=g)).clamp(0, 63)
        dt[:, 2:] = torch.maximum(dt[:, 2:], dt[:, :2] + 1)

        def masks(bx):
            m = torch.zeros(len(bx), 64, 64, dtype=torch.bool)
            for i, (x1, y1, x2, y2) in enumerate(bx.tolist()):
                m[i, y1:y2, x1:x2] = True
            return m

        lab = torch.randint(0, 2, (5,), generator=g)
        preds.append({"masks": masks(dt), "boxes": dt.float(), "scores": torch.rand(5, generator=g), "labels": lab})
        target.append({"masks": masks(gt), "boxes": gt.float(), "labels": lab})
    seg = MeanAveragePrecision(iou_type="segm")
    seg.update(preds, target)
    box = MeanAveragePrecision(iou_type="bbox")
    box.update(preds, target)
    rs, rb = seg.compute(), box.compute()
    for k in ("map", "map_50", "map_75", "mar_100"):
        assert_close(rs[k], rb[k], atol=1e-6)
    both = MeanAveragePrecision(iou_type=("bbox", "segm"))
    both.update(preds, target)
    rboth = both.compute()
    assert_close(rboth["segm_map"], rs["map"], atol=1e-6)


def _ddp_map(rank, world, preds, target):
    m = MeanAveragePrecision()
    m.update(preds[rank::world], target[rank::world])
    res = m.compute()
    # the gathered order interleaves ranks; COCO results do not depend on image order
    stats, _, _ = _oracle(preds, target)
    assert_close(res["map"], stats[0], atol=1e-6)
    assert_close(res["mar_100"], stats[8], atol=1e-6)


@pytest.mark.ddp
def test_map_ddp():
    preds, target = _random_coco(11, n_img=8)
    run_ddp(_ddp_map, preds, target)


# ------------------------------------------------------------------------------------------------ panoptic quality
def _pq_oracle(preds, target, things, stuffs, modified=False):
    """Dict-based per-sample segment matching, straight from the panoptic-quality definition."""
    things, stuffs = set(things), set(stuffs)
    void = (1 + max([0, *things, *stuffs]), 0)
    cats = {c: i for i, c in enumerate(things)}
    cats.update({c: i + len(things) for i, c in enumerate(stuffs)})
    k = len(cats)
    iou_sum, tp, fp, fn = np.zeros(k), np.zeros(k), np.zeros(k), np.zeros(k)

    def prep(x):
        out = []
        for c, i in x.reshape(x.shape[0], -1, 2).tolist()[0] if False else []:
            pass
        return out

    for pb, tb in zip(preds, target):
        def colors(x):
            cols = []
            for c, i in x.reshape(-1, 2).tolist():
                if c in stuffs:
                    cols.append((c, 0))
                elif c in things:
                    cols.append((c, i))
                else:
                    cols.append(void)
            return cols

        pc, tc = colors(pb), colors(tb)
        from collections import Counter

        pa, ta, inter = Counter(pc), Counter(tc), Counter(zip(pc, tc))
        pm, tm = set(), set()
        for (p, t), a in inter.items():
            if t == void or p[0] != t[0]:
                continue
            union = pa[p] - inter.get((p, void), 0) + ta[t] - inter.get((void, t), 0) - a
            iou = a / union
            ci = cats[t[0]]
            if (t[0] not in stuffs or not modified) and iou > 0.5:
                pm.add(p)
                tm.add(t)
                iou_sum[ci] += iou
                tp[ci] += 1
            elif modified and t[0] in stuffs and iou > 0:
                iou_sum[ci] += iou
        for t in set(ta) - tm - {void}:
            if inter.get((void, t), 0) / ta[t] <= 0.5 and not (modified and t[0] in stuffs):
                fn[cats[t[0]]] += 1
        for p in set(pa) - pm - {void}:
            if inter.get((p, void), 0) / pa[p] <= 0.5 and not (modified and p[0] in stuffs):
                fp[cats[p[0]]] += 1
        if modified:
            for t in ta:
                if t[0] in stuffs:
                    tp[cats[t[0]]] += 1
    den = tp + 0.5 * fp + 0.5 * fn
    return np.mean(iou_sum[den > 0] / den[den > 0])


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("modified", [False, True])
def test_panoptic_quality(device, modified):
    from torchmetrics_amd.detection import ModifiedPanopticQuality, PanopticQuality

    g = torch.Generator().manual_seed(3 + modified)
    things, stuffs = [0, 1, 3], [6, 7]
    # blocky segmentations so segments overlap substantially
    cat = torch.tensor([0, 1, 3, 6, 7, 9])[torch.randint(0, 6, (3, 8, 8), generator=g)]
    cat = cat.repeat_interleave(4, 1).repeat_interleave(4, 2)
    inst = torch.randint(0, 3, (3, 32, 32), generator=g)
    target = torch.stack([cat, inst], -1)
    preds = target.clone()
    noise = torch.rand(3, 32, 32, generator=g) < 0.25
    preds[..., 0] = torch.where(noise, torch.tensor([0, 1, 3, 6, 7])[torch.randint(0, 5, (3, 32, 32), generator=g)],
                                preds[..., 0])
    cls = ModifiedPanopticQuality if modified else PanopticQuality
    m = cls(things=things, stuffs=stuffs, allow_unknown_preds_category=True).to(device)
    m.update(preds[:2].to(device), target[:2].to(device))
    m.update(preds[2:].to(device), target[2:].to(device))
    assert_close(m.compute(), _pq_oracle(preds, target, things, stuffs, modified), atol=1e-9)


def _greedy_nms(boxes, scores, thr, idxs=None):
    """Plain Python greedy NMS (the torchvision rule) as the oracle."""
    order = sorted(range(len(scores)), key=lambda i: (-float(scores[i]), i))
    keep = []
    for i in order:
        ok = True
        for j in keep:
            if idxs is not None and int(idxs[i]) != int(idxs[j]):
                continue
            a, b = boxes[i].tolist(), boxes[j].tolist()
            iw = max(min(a[2], b[2]) - max(a[0], b[0]), 0.0)
            ih = max(min(a[3], b[3]) - max(a[1], b[1]), 0.0)
            inter = iw * ih
            union = (a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter
            if inter / union > thr:
                ok = False
                break
        if ok:
            keep.append(i)
    return keep


def _rand_boxes(n, g, scale=100.0):
    xy = torch.rand(n, 2, generator=g) * scale
    wh = torch.rand(n, 2, generator=g) * scale / 4 + 1
    return torch.cat([xy, xy + wh], 1)


@pytest.mark.parametrize("n", [0, 1, 7, 130])
@pytest.mark.parametrize("batched", [False, True])
def test_nms_cpu_matches_greedy_oracle(n, batched):
    from torchmetrics_amd.functional.detection import batched_nms, nms

    g = torch.Generator().manual_seed(n)
    boxes = _rand_boxes(n, g, 30.0)
    scores = torch.rand(n, generator=g)
    if n > 3:
        scores[3] = scores[1]  # a tie: lower index first
    idxs = torch.randint(0, 3, (n,), generator=g)
    got = batched_nms(boxes, scores, idxs, 0.3) if batched else nms(boxes, scores, 0.3)
    assert got.tolist() == _greedy_nms(boxes, scores, 0.3, idxs if batched else None)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 5000, 70000])
@pytest.mark.parametrize("batched", [False, True])
def test_nms_gpu_matches_cpu(n, batched):
    """HIP bitmask NMS (csrc/detection/nms.hip) vs the CPU greedy rule: chunk boundaries, ties, class-aware."""
    from torchmetrics_amd.functional.detection import batched_nms, nms

    g = torch.Generator().manual_seed(n + batched)
    boxes = _rand_boxes(n, g, 100.0 if n < 20000 else 2000.0)
    scores = torch.rand(n, generator=g)
    scores[n // 2:n // 2 + 10] = 0.5  # equal scores across a chunk boundary
    idxs = torch.randint(0, 5, (n,), generator=g)
    for thr in (0.3, 0.7):
        if batched:
            a = batched_nms(boxes.cuda(), scores.cuda(), idxs.cuda(), thr).cpu()
            b = batched_nms(boxes, scores, idxs, thr) if n <= 5000 else None
        else:
            a = nms(boxes.cuda(), scores.cuda(), thr).cpu()
            b = nms(boxes, scores, thr) if n <= 5000 else None
        if b is not None:
            assert torch.equal(a, b)
        else:  # large case: kept indices unique, score ordered, and no kept pair (same class) above the threshold
            assert len(set(a.tolist())) == len(a)
            assert torch.all(scores[a][1:] <= scores[a][:-1])
            head = a[:2000]
            kb = boxes[head].cuda()
            iou = ops.box_pairwise(kb, kb, ops.BOX_IOU).triu(1)
            if batched:
                iou = iou * (idxs[head][:, None] == idxs[head][None, :]).cuda()
            assert float(iou.max()) <= thr


@pytest.mark.parametrize("seed", [0, 1])
@pytest.mark.parametrize("precomputed", [False, True])
def test_coco_match_native_host_matches_python_oracle(seed, precomputed):
    """Native CPU matcher (csrc/detection/coco_match_host.cpp) == the plain-loop oracle, bitwise."""
    from torchmetrics_amd.ops import _cpu

    if not ops.load_native(strict=False):
        pytest.skip("native library not built")
    g = torch.Generator().manual_seed(seed)
    groups, dets, gts = 40, [], []
    det_start, det_cnt, gt_start, gt_cnt = [], [], [], []
    nd = ng = 0
    for _ in range(groups):
        dn, gn = int(torch.randint(0, 12, (1,), generator=g)), int(torch.randint(0, 8, (1,), generator=g))
        det_start.append(nd), det_cnt.append(dn), gt_start.append(ng), gt_cnt.append(gn)
        nd, ng = nd + dn, ng + gn
    xy = torch.rand(ng, 2, generator=g, dtype=torch.float64) * 100
    wh = torch.rand(ng, 2, generator=g, dtype=torch.float64) * 60 + 1
    gbox = torch.cat([xy, wh], 1)
    src = torch.randint(0, max(ng, 1), (nd,), generator=g)
    dbox = (gbox[src] if ng else torch.rand(nd, 4, dtype=torch.float64) * 50) + torch.randn(nd, 4, generator=g,
                                                                                            dtype=torch.float64) * 4
    dbox[:, 2:] = dbox[:, 2:].abs() + 1
    darea, garea = dbox[:, 2] * dbox[:, 3], gbox[:, 2] * gbox[:, 3]
    gcrowd = (torch.rand(ng, generator=g) < 0.2).to(torch.uint8)
    i32 = lambda v: torch.tensor(v, dtype=torch.int32)  # noqa: E731
    area_rng = torch.tensor([0, 1e10, 0, 1024, 1024, 3000, 3000, 1e10], dtype=torch.float64)
    thr = torch.linspace(0.5, 0.95, 10, dtype=torch.float64)
    pre = off = None
    if precomputed:
        blocks, offs, o = [], [], 0
        for d0, dn, g0, gn in zip(det_start, det_cnt, gt_start, gt_cnt):
            blocks.append(torch.rand(dn * gn, generator=g, dtype=torch.float64))
            offs.append(o)
            o += dn * gn
        pre, off = torch.cat(blocks), torch.tensor(offs, dtype=torch.int64)
    args = (dbox, darea, gbox, garea, gcrowd, i32(det_start), i32(det_cnt), i32(gt_start), i32(gt_cnt), area_rng, thr)
    native = torch.ops.tm_amd.coco_match(*args, pre, off)
    oracle = _cpu.coco_match(*args, pre, off)
    assert torch.equal(native[0], oracle[0]) and torch.equal(native[1], oracle[1])
    assert int(native[0].sum()) > 0


def test_coco_iou_matrix_matches_scalar_formula():
    from torchmetrics_amd.detection.mean_ap import _coco_iou_matrix
    from torchmetrics_amd.ops._cpu import _coco_iou

    g = torch.Generator().manual_seed(0)
    d = torch.cat([torch.rand(9, 2, generator=g) * 50, torch.rand(9, 2, generator=g) * 30 + 0.5], 1).double()
    t = torch.cat([torch.rand(7, 2, generator=g) * 50, torch.rand(7, 2, generator=g) * 30 + 0.5], 1).double()
    crowd = torch.rand(7, generator=g) < 0.3
    got = _coco_iou_matrix(d, t, crowd)
    exp = torch.tensor([[_coco_iou(a, b, bool(c)) for b, c in zip(t.tolist(), crowd.tolist())] for a in d.tolist()],
                       dtype=torch.float64)
    torch.testing.assert_close(got, exp, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("batched", [False, True])
def test_nms_native_host_matches_matrix_fallback(batched):
    from torchmetrics_amd.ops import _cpu

    if not ops.native_available():
        pytest.skip("native library not built")
    g = torch.Generator().manual_seed(9)
    boxes = _rand_boxes(700, g, 40.0)
    scores = torch.rand(700, generator=g)
    idxs = torch.randint(0, 4, (700,), generator=g) if batched else None
    assert torch.equal(ops.nms(boxes, scores, 0.45, idxs), _cpu.nms(boxes, scores, 0.45, idxs))


@pytest.mark.parametrize("backend", ["pycocotools", "faster_coco_eval"])
def test_map_many_detection_thresholds_reference_case(backend):
    """``T/unittests/detection/test_map.py:826-856``: 0.6 with faster-coco-eval, not with pycocotools."""
    preds = [{"boxes": torch.tensor([[258.0, 41.0, 606.0, 285.0]]), "scores": torch.tensor([0.536]),
              "labels": torch.tensor([0])}]
    target = [{"boxes": torch.tensor([[214.0, 41.0, 562.0, 285.0]]), "labels": torch.tensor([0])}]
    metric = MeanAveragePrecision(max_detection_thresholds=[1, 10, 1000], backend=backend)
    res = metric(preds, target)
    if backend == "pycocotools":
        assert round(res["map"].item(), 5) != 0.6
    else:
        assert round(res["map"].item(), 5) == 0.6
    assert "mar_1" in res and "mar_10" in res and "mar_1000" in res


@pytest.mark.parametrize(("box_format", "iou_val_expected", "map_val_expected"),
                         [("xyxy", 0.25, 1), ("xywh", 0.143, 0.0), ("cxcywh", 0.143, 0.0)])
def test_map_box_format_reference_case(box_format, iou_val_expected, map_val_expected):
    """``T/unittests/detection/test_map.py:686-712``: only the right box format scores 1."""
    preds = [{"boxes": torch.tensor([[0.5, 0.5, 1, 1]]), "scores": torch.tensor([1.0]), "labels": torch.tensor([0])}]
    targets = [{"boxes": torch.tensor([[0, 0, 1, 1]]), "labels": torch.tensor([0])}]
    metric = MeanAveragePrecision(box_format=box_format, iou_thresholds=[0.2], extended_summary=True)
    metric.update(preds, targets)
    result = metric.compute()
    assert result["map"].item() == map_val_expected
    assert round(float(result["ious"][(0, 0)]), 3) == iou_val_expected


@pytest.mark.gpu
def test_coco_accumulate_kernel_matches_torch_path(monkeypatch):
    """The fused accumulation kernel (csrc/detection/coco_accumulate.hip) equals the batched-torch accumulation bit
    for bit (same integer counts, same fp64 formulas), for all IoU thresholds, areas and max-dets."""
    from benchmarks.bench_map import make_data
    from torchmetrics_amd import ops
    from torchmetrics_amd.detection import MeanAveragePrecision

    dev = torch.device("cuda", 0)
    preds, target = make_data(96, dev, seed=3)

    def run():
        m = MeanAveragePrecision(class_metrics=True, extended_summary=True, max_detection_thresholds=[1, 7, 50]).to(dev)
        for i in range(0, 96, 32):
            m.update(preds[i:i + 32], target[i:i + 32])
        return m.compute()

    fused = run()
    monkeypatch.setattr(ops, "coco_accumulate", lambda *a, **k: False)
    monkeypatch.setattr(ops, "coco_accumulate_sorted", lambda *a, **k: False)
    ref = run()
    for key in ("precision", "recall", "scores", "map", "map_per_class", "mar_50_per_class", "mar_small"):
        assert torch.equal(fused[key], ref[key]), key


@pytest.mark.gpu
@pytest.mark.parametrize("score_dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("average", ["macro", "micro"])
@pytest.mark.parametrize("variant", ["plain", "int32_labels_no_area", "big_images"])
def test_coco_prepare_kernel_matches_aten_grouping(monkeypatch, score_dtype, average, variant):
    """The one-launch grouping stage (csrc/detection/coco_prepare.hip: per-image LDS ranking into (image, category,
    score) order, group tables, non-ignored ground-truth histogram) gives bit-identical precision / recall / scores and
    summary to the ATen grouping path (sorts, histograms, gathers): score ties, crowds, areas absent (box area used),
    int32 labels, empty images, images larger than a block (> 256 detections) and micro averaging (labels outside the
    category axis)."""
    from torchmetrics_amd.detection import _coco_eval

    dev = torch.device("cuda", 0)
    big = variant == "big_images"
    preds, target = _random_coco(11, n_img=10, n_cls=5, max_gt=40 if big else 8, max_det=700 if big else 15)
    preds[3] = {"boxes": torch.zeros(0, 4), "scores": torch.zeros(0), "labels": torch.zeros(0, dtype=torch.long)}
    target[5] = {"boxes": torch.zeros(0, 4), "labels": torch.zeros(0, dtype=torch.long),
                 "iscrowd": torch.zeros(0, dtype=torch.long)}
    for p in preds:
        p["scores"] = p["scores"].to(score_dtype)
        if variant == "int32_labels_no_area":
            p["labels"] = p["labels"].int()
    for t in target:
        if variant == "int32_labels_no_area":
            t["labels"] = t["labels"].int()
        else:
            t["area"] = torch.where(torch.rand(t["labels"].numel()) < 0.3, torch.zeros(t["labels"].numel()),
                                    torch.rand(t["labels"].numel()) * 9000)
    mdt = [1, 10, 300] if big else [1, 7, 50]

    def run():
        m = MeanAveragePrecision(class_metrics=True, extended_summary=True, max_detection_thresholds=mdt,
                                 average=average).to(dev)
        m.update(_to(preds[:6], dev), _to(target[:6], dev))
        m.update(_to(preds[6:], dev), _to(target[6:], dev))
        return m.compute()

    calls = []
    real = ops.coco_prepare
    monkeypatch.setattr(ops, "coco_prepare", lambda *a: calls.append(1) or real(*a))
    fused = run()
    assert calls, "the prepared path did not run"
    monkeypatch.setattr(_coco_eval, "PREP_MAX_PER_IMAGE", -1)
    ref = run()
    for key in ref:
        if key == "ious":
            continue
        assert torch.equal(fused[key], ref[key]), key


@pytest.mark.gpu
@pytest.mark.parametrize("backend,mdt", [("faster_coco_eval", [1, 7, 50]), ("pycocotools", [1, 7, 50]),
                                         ("pycocotools", [1, 10, 100])])
@pytest.mark.parametrize("average", ["macro", "micro"])
def test_coco_summary_kernel_matches_torch_reductions(monkeypatch, backend, mdt, average):
    """The one-launch summary (coco_summary_kernel: masked precision / recall sums per (t, a, m) and the per-class
    numbers) gives the same summary and per-class values as the masked torch reductions it replaced, including the
    legacy mAP at a max-dets value that is absent (-1) and micro averaging (a second, per-class evaluation)."""
    from benchmarks.bench_map import make_data
    from torchmetrics_amd import ops
    from torchmetrics_amd.detection import MeanAveragePrecision

    dev = torch.device("cuda", 0)
    preds, target = make_data(64, dev, seed=5)

    def run():
        m = MeanAveragePrecision(class_metrics=True, max_detection_thresholds=mdt, backend=backend,
                                 average=average).to(dev)
        m.update(preds[:32], target[:32])
        m.update(preds[32:], target[32:])
        return m.compute()

    fused = run()
    monkeypatch.setattr(ops, "coco_summary", lambda *a, **k: None)
    ref = run()
    assert fused.keys() == ref.keys()
    for key in fused:
        torch.testing.assert_close(fused[key].double(), ref[key].double(), rtol=1e-6, atol=1e-7, msg=key)


def _ddp_map_packed(rank, world, preds, target):
    """The per-image states cross the engine flat (Metric._packed_sync_plan); rank 1 holds one image more than rank 0
    and updates twice; after compute() the local (chunked, unbuilt) states are back; the synced order is element-major
    as the reference's per-element gather (image 0 of every rank, then image 1, ...)."""
    from torchmetrics_amd.parallel.sync import comm_stats

    mine = list(range(rank, len(preds), world)) + ([len(preds) - 1] if rank == 1 else [])
    m = MeanAveragePrecision()
    m.update([preds[i] for i in mine[:2]], [target[i] for i in mine[:2]])
    m.update([preds[i] for i in mine[2:]], [target[i] for i in mine[2:]])
    assert "_chunks" in m.__dict__ and "detection_box" in m.__dict__["_chunks"]
    comm_stats(reset=True)
    res = m.compute()
    stats = comm_stats()
    assert stats["all_gather"] <= 4, stats  # one header + one payload per dtype bucket, not one per image
    assert "detection_box" in m.__dict__["_chunks"]  # unsync restored the chunks unbuilt
    allp = [preds[i] for i in range(len(preds))] + [preds[-1]]
    allt = [target[i] for i in range(len(target))] + [target[-1]]
    stats_ref, _, _ = _oracle(allp, allt)
    assert_close(res["map"], stats_ref[0], atol=1e-6)
    assert_close(res["mar_100"], stats_ref[8], atol=1e-6)
    m.sync()
    lab = m.detection_labels
    per_rank = [list(range(r, len(preds), world)) + ([len(preds) - 1] if r == 1 else []) for r in range(world)]
    order = [per_rank[r][e] for e in range(max(map(len, per_rank))) for r in range(world) if e < len(per_rank[r])]
    assert len(lab) == len(order)
    for got, i in zip(lab, order):
        assert torch.equal(got, preds[i]["labels"])
    m.unsync()


@pytest.mark.ddp
def test_map_ddp_packed_sync():
    preds, target = _random_coco(13, n_img=9)
    run_ddp(_ddp_map_packed, preds, target)


def _map_batch(n_img, seed, box_dtype=torch.float32, drop_keys=()):
    g = torch.Generator().manual_seed(seed)
    preds, target = [], []
    for i in range(n_img):
        nd, ng = int(torch.randint(0, 12, (1,), generator=g)), int(torch.randint(0, 6, (1,), generator=g))
        xy = torch.rand(ng, 2, generator=g) * 100
        gb = torch.cat([xy, xy + torch.rand(ng, 2, generator=g) * 50 + 1], 1).to(box_dtype)
        dxy = torch.rand(nd, 2, generator=g) * 100
        db = torch.cat([dxy, dxy + torch.rand(nd, 2, generator=g) * 50 + 1], 1).to(box_dtype)
        p = {"boxes": db, "scores": torch.rand(nd, generator=g), "labels": torch.randint(0, 5, (nd,), generator=g)}
        t = {"boxes": gb, "labels": torch.randint(0, 5, (ng,), generator=g)}
        if "iscrowd" not in drop_keys or i % 2:
            t["iscrowd"] = (torch.rand(ng, generator=g) < 0.2).long()
        if "area" not in drop_keys or i % 3 == 0:
            t["area"] = torch.rand(ng, generator=g) * 1000 if "area_float" in drop_keys else torch.randint(
                1, 1000, (ng,), generator=g)
        preds.append(p)
        target.append(t)
    return preds, target


@pytest.mark.gpu
@pytest.mark.parametrize("box_format", ["xyxy", "xywh", "cxcywh"])
@pytest.mark.parametrize("drop_keys", [(), ("iscrowd",), ("iscrowd", "area")])
@pytest.mark.parametrize("box_dtype", [torch.float32, torch.float64])
def test_map_native_pack_matches_python_path(monkeypatch, box_format, drop_keys, box_dtype):
    """csrc/bindings/fastcall.cpp map_pack + csrc/detection/pack_images.hip: the flat states equal the Python
    packing (cat + box_convert), including empty images and missing iscrowd / area; compute() is identical."""
    dev = torch.device("cuda", 0)
    batches = [_map_batch(17, s, box_dtype, drop_keys) for s in range(3)]
    to = lambda b: [{k: v.to(dev) for k, v in d.items()} for d in b]  # noqa: E731
    native = MeanAveragePrecision(box_format=box_format, class_metrics=True).to(dev)
    python = MeanAveragePrecision(box_format=box_format, class_metrics=True).to(dev)
    calls = []
    real = ops.map_pack
    monkeypatch.setattr(ops, "map_pack", lambda *a: calls.append(1) or real(*a))
    for p, t in batches:
        native.update(to(p), to(t))
    assert len(calls) == 3
    monkeypatch.setattr(MeanAveragePrecision, "_native_pack", lambda self, p, t: False)
    for p, t in batches:
        python.update(to(p), to(t))
    for name in MeanAveragePrecision._NATIVE_ORDER:
        a, sa = native._packed_state(name)
        b, sb = python._packed_state(name)
        assert sa == sb, name
        assert a.dtype == b.dtype and torch.equal(a, b), name
    ra, rb = native.compute(), python.compute()
    for k in rb:
        torch.testing.assert_close(ra[k], rb[k], equal_nan=True)


@pytest.mark.gpu
def test_map_native_pack_declines_irregular_batches():
    dev = torch.device("cuda", 0)
    p, t = _map_batch(4, 9)
    p = [{k: v.to(dev) for k, v in d.items()} for d in p]
    t = [{k: v.to(dev) for k, v in d.items()} for d in t]
    assert ops.map_pack(p, t, 1) is not None
    mixed = [dict(d) for d in p]
    mixed[1]["scores"] = mixed[1]["scores"].double()
    assert ops.map_pack(mixed, t, 1) is None  # one dtype per state
    short = [dict(d) for d in p]
    short[2]["scores"] = short[2]["scores"][:-1] if short[2]["scores"].numel() else torch.rand(1, device=dev)
    assert ops.map_pack(short, t, 1) is None  # per-image lengths disagree: the Python validator raises
    with pytest.raises(ValueError):
        MeanAveragePrecision().to(dev).update(short, t)
    cpu = [{k: v.cpu() for k, v in d.items()} for d in p]
    assert ops.map_pack(cpu, [{k: v.cpu() for k, v in d.items()} for d in t], 1) is None


@pytest.mark.gpu
@pytest.mark.parametrize("dt_a,dt_b", [(torch.int64, torch.int64), (torch.int32, torch.int64), (torch.uint8, torch.int16)])
def test_small_unique_kernel_matches_torch_unique(dt_a, dt_b):
    """ops.small_unique (one-block LDS bitmap + scan, csrc/detection/coco_prepare.hip) equals torch.unique of the
    concatenation; values outside [0, 65536) or more than 4096 distinct values decline (None)."""
    g = torch.Generator().manual_seed(7)
    hi_a = 200 if dt_a == torch.uint8 else 60000
    a = torch.randint(0, hi_a, (70_000,), generator=g).to(dt_a)
    b = torch.randint(0, 3000, (513,), generator=g).to(dt_b)
    b[:5] = torch.tensor([0, 1, 2, 2, 2999], dtype=dt_b)
    a_small = a[:3000]
    ref = torch.unique(torch.cat([a_small.long(), b.long()]))
    got = ops.small_unique(a_small.cuda(), b.cuda())
    assert got is not None
    assert got[0] == ref.tolist() and torch.equal(got[1].cpu(), ref)
    if dt_a != torch.uint8:
        assert ops.small_unique(a.cuda(), b.cuda()) is None  # > 4096 distinct values
    neg = b.clone()
    neg[7] = -1 if dt_b != torch.uint8 else 0
    if dt_b != torch.uint8:
        assert ops.small_unique(a_small.cuda(), neg.cuda()) is None  # outside the range
    assert ops.small_unique(a_small, b) is None  # CPU
