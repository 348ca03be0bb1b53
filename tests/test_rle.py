"""Run-length encoded masks (``csrc/detection/rle.hip``, ``detection/_rle.py``) and the mAP segm path built on them.

Oracles: dense numpy masks (IoU = pixel counts), the plain-Python COCO evaluator (``tests/_coco_oracle.py``) with a
dense-mask IoU, and COCO's documented RLE conventions (column-major runs, background first).  pycocotools is not
installable here, so byte-for-byte parity of the compressed strings / polygon rasteriser with it is unpinned beyond
the properties tested below (round trips, rectangle polygons covering exactly their pixel block).
"""
import json

import numpy as np
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.detection import MeanAveragePrecision
from torchmetrics_amd.detection import _rle
from tests._coco_oracle import coco_eval, summarize
from tests.helpers import assert_close, run_ddp

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
IOU_THRS = torch.linspace(0.5, 0.95, 10).tolist()
REC_THRS = torch.linspace(0.0, 1.0, 101).tolist()


def _blobs(g, n, h, w, noise=0.0):
    """Random ellipses / rectangles (+ optional salt noise): realistic run structure with edge cases."""
    yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    out = torch.zeros(n, h, w, dtype=torch.bool)
    for i in range(n):
        cy, cx = torch.rand(2, generator=g) * torch.tensor([h, w])
        ry, rx = torch.rand(2, generator=g) * torch.tensor([h, w]) * 0.4 + 1
        if i % 3 == 0:
            out[i] = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1
        else:
            out[i] = ((yy - cy).abs() <= ry) & ((xx - cx).abs() <= rx)
    if noise:
        out ^= torch.rand(n, h, w, generator=g) < noise
    return out


SHAPES = [(3, 1, 1), (4, 1, 37), (4, 29, 1), (5, 17, 23), (3, 40, 300), (2, 64, 513), (0, 8, 8)]


def _edge_masks(h, w):
    full = torch.ones(1, h, w, dtype=torch.bool)
    empty = torch.zeros(1, h, w, dtype=torch.bool)
    first = torch.zeros(1, h, w, dtype=torch.bool)
    first[0, 0, 0] = True
    last = torch.zeros(1, h, w, dtype=torch.bool)
    last[0, -1, -1] = True
    return torch.cat([full, empty, first, last])


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("aligned", [False, True])
def test_encode_matches_contract_and_decodes(device, aligned):
    g = torch.Generator().manual_seed(0)
    if aligned:  # every row 4-byte aligned: the 4-column kernels; W > 1024 exercises the tile carry
        masks = [_blobs(g, n, h, w, noise=0.02) for n, h, w in [(3, 40, 300), (2, 17, 516), (2, 9, 1028), (1, 1, 4)]]
        masks += [_edge_masks(9, 300), (torch.rand(2, 6, 8, generator=g) < 0.5).to(torch.uint8) * 255]
    else:
        masks = [_blobs(g, n, h, w, noise=0.02 if h > 1 else 0.3) for n, h, w in SHAPES]
        masks += [_edge_masks(9, 300), torch.zeros(2, 5, 6, dtype=torch.uint8)]
    dev_masks = [m.to(device) for m in masks]
    packs = ops.rle_encode(dev_masks)
    want = ops._cpu.rle_encode(masks)
    assert len(packs) == len(masks)
    for p, wnt, m in zip(packs, want, masks):
        assert p.device.type == device and p.dtype == torch.int32
        assert torch.equal(p.cpu(), wnt), (m.shape, p[:12], wnt[:12])
        assert torch.equal(_rle.decode(p).cpu(), m.bool())
        n = m.shape[0]
        assert torch.equal(p[3:3 + n].cpu().long(), m.flatten(1).ne(0).sum(1))


def test_contract_matches_coco_counts_convention():
    # 2x3 mask, column-major order: (0,0)=1 (1,0)=0 | (0,1)=0 (1,1)=1 | (0,2)=1 (1,2)=1
    m = torch.tensor([[[1, 0, 1], [0, 1, 1]]], dtype=torch.bool)
    pack = ops.rle_encode([m])[0].tolist()
    n, h, w = pack[:3]
    assert (n, h, w) == (1, 2, 3)
    pos = pack[4 + 2 * n:]
    counts = _rle.positions_to_counts(pos, h * w)
    assert counts == [0, 1, 2, 3]  # COCO: background run first (0 here), then alternating
    assert _rle.counts_to_positions(counts) == pos


@pytest.mark.parametrize("seed", range(4))
def test_counts_string_roundtrip(seed):
    rng = np.random.default_rng(seed)
    counts = [int(rng.integers(0, 3))] + rng.integers(1, 5000, size=int(rng.integers(1, 60))).tolist()
    s = _rle.counts_to_string(counts)
    assert all(48 <= ord(c) < 48 + 64 for c in s)
    assert _rle.string_to_counts(s) == counts


def test_segmentation_formats_agree():
    g = torch.Generator().manual_seed(3)
    m = _blobs(g, 1, 31, 45, noise=0.05)[0]
    pack = ops.rle_encode([m[None]])[0]
    coco = _rle.pack_to_coco(pack)[0]
    assert coco["size"] == [31, 45]
    dense = _rle.segmentation_to_mask(coco, 31, 45)
    assert np.array_equal(dense, m.numpy().astype(np.uint8))
    raw = {"size": [31, 45], "counts": _rle.string_to_counts(coco["counts"])}
    assert np.array_equal(_rle.segmentation_to_mask(raw, 31, 45), dense)


def test_polygon_rectangle_covers_its_pixel_block():
    mask = _rle.segmentation_to_mask([[2, 3, 12, 3, 12, 9, 2, 9]], 20, 16)
    ref = np.zeros((20, 16), dtype=np.uint8)
    ref[3:9, 2:12] = 1
    assert np.array_equal(mask, ref)


def test_polygon_triangle_close_to_pixel_centre_test():
    h, w = 50, 60
    tri = [5.0, 5.0, 55.0, 10.0, 20.0, 45.0]
    mask = _rle.segmentation_to_mask([tri], h, w).astype(bool)
    yy, xx = np.mgrid[0:h, 0:w]
    (x0, y0), (x1, y1), (x2, y2) = np.array(tri).reshape(3, 2)

    def side(ax, ay, bx, by):
        return (bx - ax) * (yy - ay) - (by - ay) * (xx - ax)

    s0, s1, s2 = side(x0, y0, x1, y1), side(x1, y1, x2, y2), side(x2, y2, x0, y0)
    inside = ((s0 >= 0) & (s1 >= 0) & (s2 >= 0)) | ((s0 <= 0) & (s1 <= 0) & (s2 <= 0))
    iou = (mask & inside).sum() / (mask | inside).sum()
    assert iou > 0.9


def _dense_iou(d, g, crowd):
    inter = np.logical_and(d, g).sum()
    if inter == 0:
        return 0.0
    union = d.sum() if crowd else d.sum() + g.sum() - inter
    return inter / union


@pytest.mark.parametrize("device", DEVICES)
def test_rle_iou_matches_dense(device):
    g = torch.Generator().manual_seed(1)
    dm = [_blobs(g, 6, 40, 70, noise=0.01), _blobs(g, 3, 33, 21)]
    gm = [_blobs(g, 4, 40, 70), _blobs(g, 2, 33, 21, noise=0.01), torch.zeros(0, 12, 12, dtype=torch.bool)]
    dev = torch.device(device)
    dbuf, ddesc = _rle.descriptors(ops.rle_encode([m.to(dev) for m in dm]), [6, 3], dev)
    gbuf, gdesc = _rle.descriptors(ops.rle_encode([m.to(dev) for m in gm]), [4, 2, 0], dev)
    d_all = [m for x in dm for m in x]
    g_all = [m for x in gm for m in x]
    crowd = torch.tensor([0, 1, 0, 0, 1, 0], dtype=torch.uint8)
    pd = torch.arange(len(d_all)).repeat_interleave(len(g_all))
    pg = torch.arange(len(g_all)).repeat(len(d_all))
    out = ops.rle_iou(dbuf, ddesc, gbuf, gdesc, pd.to(dev), pg.to(dev), crowd.to(dev)).cpu()
    for p in range(pd.numel()):
        d, gg = d_all[pd[p]], g_all[pg[p]]
        exp = -1.0 if d.shape != gg.shape else _dense_iou(d.numpy(), gg.numpy(), bool(crowd[pg[p]]))
        assert abs(float(out[p]) - exp) < 1e-12, (p, float(out[p]), exp)
    py = ops._cpu.rle_iou(dbuf.cpu(), ddesc.cpu(), gbuf.cpu(), gdesc.cpu(), pd, pg, crowd)
    assert_close(out, py, atol=0, rtol=0)


def _segm_inputs(seed, n_img=5, n_cls=3, h=48, w=64):
    g = torch.Generator().manual_seed(seed)
    preds, target = [], []
    for _ in range(n_img):
        ng = int(torch.randint(1, 6, (1,), generator=g))
        gt = _blobs(g, ng, h, w)
        gl = torch.randint(0, n_cls, (ng,), generator=g)
        nd = int(torch.randint(0, 8, (1,), generator=g))
        src = torch.randint(0, ng, (nd,), generator=g)
        # detections: ground truths shifted by a few pixels with some flipped pixels, plus clutter
        dm = torch.roll(gt[src], shifts=(int(torch.randint(-3, 4, (1,), generator=g)),), dims=(2,))
        dm ^= torch.rand(dm.shape, generator=g) < 0.01
        if nd > 2:
            dm[-1] = _blobs(g, 1, h, w)[0]
        dl = torch.where(torch.rand(nd, generator=g) < 0.2, torch.randint(0, n_cls, (nd,), generator=g), gl[src])
        preds.append({"masks": dm, "scores": (torch.rand(nd, generator=g) * 10).round() / 10, "labels": dl})
        target.append({"masks": gt, "labels": gl, "iscrowd": (torch.rand(ng, generator=g) < 0.2).long()})
    return preds, target


def _segm_oracle(preds, target):
    cats = sorted(set(torch.cat([p["labels"] for p in preds] + [t["labels"] for t in target]).tolist()))
    dets = [[(m.numpy(), s, c) for m, s, c in zip(p["masks"], p["scores"].tolist(), p["labels"].tolist())]
            for p in preds]
    gts = [[(m.numpy(), c, cr, float(m.sum())) for m, c, cr in zip(t["masks"], t["labels"].tolist(),
                                                                   t["iscrowd"].tolist())] for t in target]
    prec, rec = coco_eval(dets, gts, cats, IOU_THRS, REC_THRS, [1, 10, 100], iou_fn=_dense_iou,
                          area_fn=lambda m: float(m.sum()))
    return summarize(prec, rec, IOU_THRS, [1, 10, 100]), prec, rec


def _to(items, device):
    return [{k: v.to(device) for k, v in it.items()} for it in items]


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("seed", [0, 1])
def test_map_segm_vs_dense_mask_oracle(device, seed):
    preds, target = _segm_inputs(seed)
    m = MeanAveragePrecision(iou_type="segm", extended_summary=True, class_metrics=True).to(device)
    m.update(_to(preds[:2], device), _to(target[:2], device))
    m.update(_to(preds[2:], device), _to(target[2:], device))
    res = m.compute()
    stats, prec, rec = _segm_oracle(preds, target)
    names = ["map", "map_50", "map_75", "map_small", "map_medium", "map_large", "mar_1", "mar_10", "mar_100",
             "mar_small", "mar_medium", "mar_large"]
    for name, v in zip(names, stats):
        assert_close(res[name], v, atol=1e-6)
    assert_close(res["precision"], prec, atol=1e-6)
    assert_close(res["recall"], rec, atol=1e-6)
    # extended-summary IoU matrices from the runs equal dense IoUs
    for (img, cls), mat in res["ious"].items():
        dl = preds[img]["labels"] == cls
        gl = target[img]["labels"] == cls
        order = torch.argsort(-preds[img]["scores"][dl], stable=True)
        dms = preds[img]["masks"][dl][order]
        gms = target[img]["masks"][gl]
        crowd = target[img]["iscrowd"][gl]
        exp = torch.tensor([[_dense_iou(d.numpy(), gg.numpy(), bool(c)) for gg, c in zip(gms, crowd)] for d in dms])
        assert_close(mat, exp.reshape(mat.shape).float(), atol=1e-6)


def test_segm_state_is_run_length_sized():
    g = torch.Generator().manual_seed(2)
    masks = _blobs(g, 20, 480, 640)
    m = MeanAveragePrecision(iou_type="segm")
    m.update([{"masks": masks, "scores": torch.rand(20, generator=g), "labels": torch.zeros(20, dtype=torch.long)}],
             [{"masks": masks[:5], "labels": torch.zeros(5, dtype=torch.long)}])
    state_bytes = sum(p.numel() * p.element_size() for p in m.detection_mask + m.groundtruth_mask)
    dense_bytes = 25 * 480 * 640
    assert state_bytes * 50 < dense_bytes, (state_bytes, dense_bytes)
    assert float(m.compute()["map"]) > 0


def _ddp_segm(rank, world):
    preds, target = _segm_inputs(4, n_img=6)
    m = MeanAveragePrecision(iou_type="segm")
    m.update(preds[rank::world], target[rank::world])
    res = m.compute()
    stats, _, _ = _segm_oracle(preds, target)
    assert_close(res["map"], stats[0], atol=1e-6)
    assert_close(res["mar_100"], stats[8], atol=1e-6)


def test_map_segm_ddp():
    run_ddp(_ddp_segm)


@pytest.mark.parametrize("iou_type", ["segm", ("bbox", "segm")])
def test_coco_json_roundtrip_segm(tmp_path, iou_type):
    preds, target = _segm_inputs(5, n_img=4)
    if "bbox" in iou_type:
        for p in preds + target:
            m = p["masks"]
            boxes = []
            for mk in m:
                ys, xs = torch.nonzero(mk, as_tuple=True)
                boxes.append([xs.min(), ys.min(), xs.max() + 1, ys.max() + 1] if ys.numel() else [0, 0, 1, 1])
            p["boxes"] = torch.tensor(boxes, dtype=torch.float32).reshape(-1, 4)
    m = MeanAveragePrecision(iou_type=iou_type)
    m.update(preds, target)
    base = str(tmp_path / "rt")
    m.tm_to_coco(base)
    with open(f"{base}_target.json") as f:
        tj = json.load(f)
    assert all(isinstance(a["segmentation"]["counts"], str) for a in tj["annotations"])
    bp, bt = MeanAveragePrecision.coco_to_tm(f"{base}_preds.json", f"{base}_target.json", iou_type=iou_type)
    for p, q in zip(bp, preds):
        assert torch.equal(p["masks"].bool(), q["masks"].bool())
    for t, q in zip(bt, target):
        assert torch.equal(t["masks"].bool(), q["masks"].bool())
    m2 = MeanAveragePrecision(iou_type=iou_type)
    m2.update(bp, bt)
    r1, r2 = m.compute(), m2.compute()
    for k in r1:
        if k != "classes":
            assert_close(r2[k], r1[k], atol=1e-6)


def test_coco_to_tm_polygons(tmp_path):
    gt = {"images": [{"id": 7, "height": 20, "width": 16}],
          "annotations": [{"id": 1, "image_id": 7, "category_id": 1, "iscrowd": 0, "area": 60.0, "bbox": [2, 3, 10, 6],
                           "segmentation": [[2, 3, 12, 3, 12, 9, 2, 9]]}],
          "categories": [{"id": 1, "name": "a"}]}
    dt = [{"image_id": 7, "category_id": 1, "score": 0.9, "bbox": [2, 3, 10, 6],
           "segmentation": {"size": [20, 16], "counts": _rle.counts_to_string([63, 6, 14, 6, 231])}}]
    (tmp_path / "t.json").write_text(json.dumps(gt))
    (tmp_path / "p.json").write_text(json.dumps(dt))
    bp, bt = MeanAveragePrecision.coco_to_tm(str(tmp_path / "p.json"), str(tmp_path / "t.json"), iou_type="segm")
    assert bt[0]["masks"].shape == (1, 20, 16) and int(bt[0]["masks"].sum()) == 60
    assert int(bp[0]["masks"].sum()) == 12
