"""GPU COCO evaluation (evaluate + accumulate + summarize) for ``MeanAveragePrecision``.

Behavioural reference: pycocotools ``COCOeval`` as driven by ``S/detection/mean_ap.py:513-588`` (parameters
``iouThrs``, ``recThrs``, ``maxDets``, the 4 default area ranges, per (image, category) greedy matching, per
(category, area, max-dets) precision / recall accumulation, the 12-number summary).

MI355X design: every step is a batched device computation over *all* images and categories at once --
(1) one radix sort of (group, descending score) keys groups detections by (image, category) in score order, device
histograms give the group sizes (the largest max-dets value truncates each group in place: no compaction, no host
sync); (2) the ``coco_match`` HIP kernel runs every (group, area range, IoU threshold) greedy matching problem in its
own thread; (3) accumulation: on ROCm the matcher's flags are packed into true / false positive bit words and one
wave per (category, IoU threshold, area, max-dets) sweeps the category's score-sorted detections with ballot counts
and a suffix-max envelope, ``csrc/detection/coco_accumulate.hip``; elsewhere a segmented cumulative sum over
detections sorted by (category, score) for all thresholds / areas at once, a segmented reverse running-max for the
envelope and one ``searchsorted`` + scatter per max-dets; (4) the summary is four masked reductions crossing to the
host in one transfer.
"""
from itertools import accumulate
from typing import Dict, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_amd import ops

AREA_RANGES = ((0.0, 1e5**2), (0.0, 32.0**2), (32.0**2, 96.0**2), (96.0**2, 1e5**2))

# device copies of the configuration constants (IoU / recall thresholds, area ranges), made once per (device, values):
# a ``torch.tensor(..., device=dev)`` from host memory is a synchronous copy that drains the stream, so three of them
# per compute() kept the host from running ahead of the device
_CONST: Dict[Tuple[torch.device, Tuple[float, ...]], Tensor] = {}


def _device_const(values: Sequence, dev: torch.device) -> Tensor:
    key = (dev, tuple(float(v) for v in values))
    t = _CONST.get(key)
    if t is None:
        if len(_CONST) > 64:
            _CONST.clear()
        t = _CONST[key] = torch.tensor(key[1], dtype=torch.float64, device=dev)
    return t


def _to_device_async(values: List[int], dev: torch.device) -> Tensor:
    """int64 host values on ``dev`` without draining the stream: a pinned staging buffer and a non-blocking copy (a
    pageable source makes the copy wait for the device's queue)."""
    t = torch.tensor(values, dtype=torch.long)
    if dev.type == "cpu":
        return t
    return t.pin_memory().to(dev, non_blocking=True)


AREA_LABELS = ("all", "small", "medium", "large")
PREP_MAX_PER_IMAGE = 2048  # csrc/detection/coco_prepare.hip kPrepMaxPerImage


def _segment_starts(sorted_keys: Tensor) -> Tensor:
    """Index of the first element of each element's run of equal keys."""
    n = sorted_keys.numel()
    idx = torch.arange(n, device=sorted_keys.device)
    start = torch.ones(n, dtype=torch.bool, device=sorted_keys.device)
    if n > 1:
        start[1:] = sorted_keys[1:] != sorted_keys[:-1]
    return torch.where(start, idx, torch.zeros_like(idx)).cummax(0).values


def _desc_key32(x: Tensor) -> Tensor:
    """int64 in [0, 2^32): larger for smaller ``x``, ties equal -- the f32 bit pattern made order-preserving (sign
    flip for positives, full flip for negatives) and reversed; -0 is +0 and NaN sorts last, as in
    ``argsort(-x)``."""
    xf = x.float() + 0.0  # (-0.0 + 0.0 = +0.0)
    b = xf.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    ordered = torch.where(b >= 0x80000000, 0xFFFFFFFF - b, b | 0x80000000)  # ascending in x
    return torch.where(torch.isnan(xf), 0xFFFFFFFF, 0xFFFFFFFF - ordered)


def _group_score_order(group: Tensor, score: Tensor, desc32: Optional[Tensor]) -> Tensor:
    """Permutation sorting by (group ascending, score descending), ties in input order (stable) -- what
    ``argsort(-score, stable)`` then ``argsort(group[.], stable)`` give."""
    if desc32 is not None and group.numel() < (1 << 31):
        return torch.sort((group << 32) | desc32, stable=True).indices
    order = torch.argsort(-score, stable=True)
    return order[torch.argsort(group[order], stable=True)]


class Packed:
    """A per-image list state held flat: ``flat`` = the images' tensors back to back along dim 0, ``sizes`` = each
    image's row count (``Metric._packed_state``).  ``len()`` is the number of images; :func:`cat_states` and
    :func:`image_sizes` read it without per-image tensors."""

    __slots__ = ("flat", "sizes")

    def __init__(self, flat: Tensor, sizes: List[int]) -> None:
        self.flat, self.sizes = flat, sizes

    def __len__(self) -> int:
        return len(self.sizes)

    def zeros_like(self) -> "Packed":
        return Packed(torch.zeros_like(self.flat), self.sizes)


def image_sizes(seq: Union[Sequence[Tensor], Packed]) -> List[int]:
    """Per-image element counts of a 1-D-per-image list state (labels, scores, ...)."""
    if isinstance(seq, Packed):
        return seq.sizes
    return [x.numel() for x in seq]


def cat_states(seq: Union[Sequence[Tensor], Packed], dev: torch.device, shape_tail: Tuple[int, ...] = ()) -> Tensor:
    """Concatenate per-image list states into one ``[N, *shape_tail]`` tensor on ``dev``: one ``cat`` when they already
    have that layout on one device (no per-image Python work), else reshaped one by one."""
    if isinstance(seq, Packed):
        out = seq.flat.to(dev)
        return out if tuple(out.shape[1:]) == tuple(shape_tail) else out.reshape(-1, *shape_tail)
    seq = seq if isinstance(seq, list) else list(seq)
    if not seq:
        return torch.zeros((0, *shape_tail), device=dev)
    try:
        out = torch.cat(seq)
        if out.dim() == 1 + len(shape_tail) and tuple(out.shape[1:]) == tuple(shape_tail):
            return out.to(dev)
    except RuntimeError:
        pass
    return torch.cat([x.to(device=dev).reshape(-1, *shape_tail) for x in seq])


def coco_evaluate(
    det_boxes: Sequence[Tensor],
    det_scores: Sequence[Tensor],
    det_labels: Sequence[Tensor],
    gt_boxes: Sequence[Tensor],
    gt_labels: Sequence[Tensor],
    gt_crowds: Sequence[Tensor],
    gt_areas: Sequence[Tensor],
    iou_thresholds: Sequence[float],
    rec_thresholds: Sequence[float],
    max_dets: Sequence[int],
    classes: Tensor,
    det_rle: Optional[Tuple[Tensor, Tensor]] = None,
    gt_rle: Optional[Tuple[Tensor, Tensor]] = None,
) -> Dict[str, Tensor]:
    """COCO precision ``[T, R, K, A, M]``, recall ``[T, K, A, M]`` and scores.

    Boxes are xywh.  With ``det_rle`` / ``gt_rle`` (``(buffer, descriptors)`` of the run-length encoded masks, one
    descriptor row per annotation in flat image order, :func:`torchmetrics_amd.detection._rle.descriptors`) IoUs are
    mask IoUs and areas are mask areas (``segm``).  ``classes`` are the sorted category ids of the K axis; annotations whose label is not
    among them are dropped (pycocotools ``catIds`` filtering).
    """
    dev = classes.device
    n_img = len(det_labels)
    t_thr = _device_const(iou_thresholds, dev)
    r_thr = _device_const(rec_thresholds, dev)
    areas = _device_const([a for r in AREA_RANGES for a in r], dev).reshape(-1, 2)
    T, R, A, M, K = t_thr.numel(), r_thr.numel(), areas.shape[0], len(max_dets), classes.numel()
    # (every entry is written below: by the accumulation kernel, which also writes -1 for categories without a
    # non-ignored ground truth, or by the torch path and the final mask)
    precision = torch.empty((T, R, K, A, M), dtype=torch.float64, device=dev)
    recall = torch.empty((T, K, A, M), dtype=torch.float64, device=dev)
    scores_out = torch.empty((T, R, K, A, M), dtype=torch.float64, device=dev)
    if K == 0:
        return {"precision": precision, "recall": recall, "scores": scores_out}

    def flat(seq, dtype, shape_tail=()):
        return cat_states(seq, dev, shape_tail).to(dtype)

    # Every step below is sync-free: no boolean-mask compaction (annotations outside the category axis and detections
    # past the largest max-dets value stay in the arrays with a sentinel group / rank and are skipped by the kernels),
    # group sizes from the device histogram (``ops.histogram``: no host max like ``torch.bincount``), ranks from the
    # group starts (no segmented cummax), and the image index expansion with a host-known output size.
    d_sizes, g_sizes = image_sizes(det_labels), image_sizes(gt_labels)
    n_det, n_gt = int(sum(d_sizes)), int(sum(g_sizes))
    if det_rle is None and dev.type == "cuda":
        fast = _evaluate_prepared(det_boxes, det_scores, det_labels, gt_boxes, gt_labels, gt_crowds, gt_areas, d_sizes,
                                  g_sizes, classes, t_thr, r_thr, areas, max_dets, precision, recall, scores_out)
        if fast:
            return {"precision": precision, "recall": recall, "scores": scores_out}
    img_ids = torch.arange(n_img, device=dev)
    sizes_dev = _to_device_async(list(d_sizes) + list(g_sizes), dev)  # one pinned, non-blocking copy for both
    d_img = torch.repeat_interleave(img_ids, sizes_dev[:n_img], output_size=n_det)
    g_img = torch.repeat_interleave(img_ids, sizes_dev[n_img:], output_size=n_gt)
    d_lab, g_lab = flat(det_labels, torch.long), flat(gt_labels, torch.long)
    d_cls = torch.searchsorted(classes, d_lab).clamp(max=K - 1)
    g_cls = torch.searchsorted(classes, g_lab).clamp(max=K - 1)
    keep_d, keep_g = classes[d_cls] == d_lab, classes[g_cls] == g_lab
    segm = det_rle is not None
    if segm:
        d_box = torch.zeros(d_lab.numel(), 4, dtype=torch.float64, device=dev)
        g_box = torch.zeros(g_lab.numel(), 4, dtype=torch.float64, device=dev)
        d_area = det_rle[1][:, 2].to(torch.float64)
        g_mask_area = gt_rle[1][:, 2].to(torch.float64)
    else:
        d_box, g_box = flat(det_boxes, torch.float64, (4,)), flat(gt_boxes, torch.float64, (4,))
        d_area = d_box[:, 2] * d_box[:, 3]
        g_mask_area = g_box[:, 2] * g_box[:, 3]
    d_score_raw = cat_states(det_scores, dev)
    d_score = d_score_raw.to(torch.float64)
    # descending-score sort keys: 32-bit scores (the usual f32 / f16 / bf16) map to an order-preserving uint32, so
    # (group, -score) is ONE int64 radix key per sort instead of two stable sorts; fp64 scores keep the two sorts
    desc32 = _desc_key32(d_score_raw) if d_score_raw.dtype in (torch.float32, torch.float16, torch.bfloat16) else None
    g_crowd_all = flat(gt_crowds, torch.long).clamp(0, 1).to(torch.uint8)
    g_area_in = flat(gt_areas, torch.float64)
    g_area = torch.where(g_area_in > 0, g_area_in, g_mask_area)
    g_crowd = g_crowd_all
    n_groups = n_img * K
    # annotations outside the category axis (micro averaging relabels everything to 0): sentinel group n_groups
    d_group = torch.where(keep_d, d_img * K + d_cls, n_groups)
    g_group = torch.where(keep_g, g_img * K + g_cls, n_groups)

    # (1) detections grouped by (image, category), score-descending (stable); each group's first max_dets[-1] are
    # matched (the rest keep their slots, with a rank the accumulation skips)
    order = _group_score_order(d_group, d_score, desc32)
    grp_s = d_group[order]
    det_cnt_all = ops.histogram(grp_s, n_groups)  # (sentinel keys skipped)
    det_start = torch.cumsum(det_cnt_all, 0) - det_cnt_all
    valid_s = grp_s < n_groups
    big = torch.iinfo(torch.int64).max // 2
    rank = torch.where(valid_s, torch.arange(order.numel(), device=dev) - det_start[grp_s.clamp(max=n_groups - 1)],
                       big)
    det_cnt = det_cnt_all.clamp(max=max_dets[-1])
    g_order = torch.argsort(g_group, stable=True)
    gt_cnt = ops.histogram(g_group, n_groups)
    gt_start = torch.cumsum(gt_cnt, 0) - gt_cnt
    d_idx = torch.arange(d_lab.numel(), device=dev)
    g_idx = torch.arange(g_lab.numel(), device=dev)

    # (2) greedy matching for every (group, area range, IoU threshold)
    pre, off = None, None
    if segm:
        pre, off = _rle_iou_blocks(det_rle, gt_rle, g_crowd_all, d_idx[order], g_idx[g_order], grp_s, rank,
                                   max_dets[-1], det_cnt, gt_start, gt_cnt, n_groups)
    dt_match, dt_ig = ops.coco_match(
        d_box[order].contiguous(), d_area[order].contiguous(), g_box[g_order].contiguous(),
        g_area[g_order].contiguous(), g_crowd[g_order].contiguous(), det_start.int(), det_cnt.int(),
        gt_start.int(), gt_cnt.int(), areas.reshape(-1).contiguous(), t_thr, pre, off)

    # (3) accumulate: detections of each category in score order (ties: image, then rank -- pycocotools mergesort);
    # sentinel detections sort into a last category K that no kernel reads
    cls_k = torch.where(valid_s, d_cls[order], K)
    score_k = d_score[order]
    o = _group_score_order(cls_k, score_k, desc32[order] if desc32 is not None else None)
    cls_s, rank_s, score_s = cls_k[o], rank[o], score_k[o]
    g_ig = (g_crowd.bool()[None, :] | (g_area[None, :] < areas[:, :1]) | (g_area[None, :] > areas[:, 1:]))  # [A, G]
    # non-ignored ground truths per (area, category): one device histogram (an fp64 index_add here serialised on
    # 80 addresses: 0.37 ms)
    key = torch.where(~g_ig & keep_g[None, :], torch.arange(A, device=dev)[:, None] * K + g_cls[None, :], -1)
    npig = ops.histogram(key.reshape(-1), A * K).reshape(A, K).to(torch.float64)
    has_gt = npig > 0
    n = cls_s.numel()
    # ROCm: one wave per (category, threshold, area, max-dets), csrc/detection/coco_accumulate.hip
    done = bool(n) and ops.coco_accumulate(dt_match, dt_ig, o, rank_s, score_s, cls_s, npig, r_thr, max_dets,
                                           precision, recall, scores_out)
    if n and not done:
        # (the batched torch path) the sentinel detections go: every segment below is a real category
        match = dt_match[..., o].bool()
        ig = dt_ig[..., o].bool()
        tp_all, fp_all = match & ~ig, ~match & ~ig  # [T, A, D]
        sel = cls_s < K
        cls_s, rank_s, score_s = cls_s[sel], rank_s[sel], score_s[sel]
        tp_all, fp_all = tp_all[..., sel], fp_all[..., sel]
        n = cls_s.numel()
    if n and not done:
        seg_first = _segment_starts(cls_s)
        is_last = torch.ones(n, dtype=torch.bool, device=dev)
        is_last[:-1] = cls_s[1:] != cls_s[:-1]
        seg_id = torch.cumsum((torch.arange(n, device=dev) == seg_first).long(), 0) - 1
        npig_d = npig[:, cls_s].clamp(min=1)[None]  # [1, A, D]
        eps = torch.finfo(torch.float64).eps
        for mi, md in enumerate(max_dets):
            incl = (rank_s < md)[None, None]
            tp_c = torch.cumsum((tp_all & incl).to(torch.float64), -1)
            fp_c = torch.cumsum((fp_all & incl).to(torch.float64), -1)
            base_tp = torch.where(seg_first > 0, tp_c[..., (seg_first - 1).clamp(min=0)], torch.zeros_like(tp_c))
            base_fp = torch.where(seg_first > 0, fp_c[..., (seg_first - 1).clamp(min=0)], torch.zeros_like(fp_c))
            tp_c, fp_c = tp_c - base_tp, fp_c - base_fp
            rc = tp_c / npig_d
            pr = tp_c / (tp_c + fp_c + eps)
            # precision envelope: running max from the end of each category segment
            off = 2.0 * (seg_id[-1] - seg_id).to(torch.float64)
            env = (pr.flip(-1) + off.flip(-1)).cummax(-1).values.flip(-1) - off
            # recall thresholds in (rc of the previous included detection, rc] belong to this detection
            inc = (rank_s < md).long()
            inc_cs = torch.cumsum(inc, 0)
            inc_before = inc_cs - inc - torch.where(seg_first > 0, inc_cs[(seg_first - 1).clamp(min=0)],
                                                    torch.zeros_like(inc_cs))
            prev_rc = torch.cat([torch.full_like(rc[..., :1], -1.0), rc[..., :-1]], -1)
            prev_rc = torch.where(inc_before > 0, prev_rc, torch.full_like(rc, -1.0))
            lo = torch.searchsorted(r_thr, prev_rc.reshape(-1, n).contiguous(), right=True).reshape(rc.shape)
            hi = torch.searchsorted(r_thr, rc.reshape(-1, n).contiguous(), right=True).reshape(rc.shape)
            nonempty = (hi > lo) & (inc > 0)
            # first recall threshold index of every non-empty range -> detection index, filled forward along R
            mark = torch.full((T, A, K, R + 1), -1, dtype=torch.long, device=dev)
            ti, ai, di = torch.nonzero(nonempty, as_tuple=True)
            mark.index_put_((ti, ai, cls_s[di], lo[ti, ai, di]), di, accumulate=False)
            mark = mark[..., :R].cummax(-1).values
            # thresholds beyond the last recall of the category get no detection
            last_idx = torch.nonzero(is_last).flatten()
            hi_last = torch.zeros(T, A, K, dtype=torch.long, device=dev)
            hi_last[..., cls_s[last_idx]] = hi[..., last_idx]
            valid = (mark >= 0) & (torch.arange(R, device=dev) < hi_last[..., None])
            safe = mark.clamp(min=0)
            q = torch.where(valid, torch.gather(env, -1, safe.reshape(T, A, -1)).reshape(T, A, K, R),
                            torch.zeros((), dtype=torch.float64, device=dev))
            ss = torch.where(valid, score_s[safe], torch.zeros((), dtype=torch.float64, device=dev))
            rec = torch.zeros(T, A, K, dtype=torch.float64, device=dev)
            rec[..., cls_s[last_idx]] = rc[..., last_idx]
            precision[..., mi] = q.permute(0, 3, 2, 1)
            scores_out[..., mi] = ss.permute(0, 3, 2, 1)
            recall[..., mi] = rec.permute(0, 2, 1)
    elif not done:
        precision.zero_()
        scores_out.zero_()
        recall.zero_()
    if not done:
        # categories without any non-ignored ground truth stay at -1 (pycocotools skips them; the kernel writes these
        # itself)
        missing = ~has_gt.T  # [K, A]
        precision.masked_fill_(missing[None, None, :, :, None], -1.0)
        scores_out.masked_fill_(missing[None, None, :, :, None], -1.0)
        recall.masked_fill_(missing[None, :, :, None], -1.0)
    return {"precision": precision, "recall": recall, "scores": scores_out}


def _evaluate_prepared(det_boxes, det_scores, det_labels, gt_boxes, gt_labels, gt_crowds, gt_areas,
                       d_sizes: List[int], g_sizes: List[int], classes: Tensor, t_thr: Tensor, r_thr: Tensor,
                       areas: Tensor, max_dets: Sequence[int], precision: Tensor, recall: Tensor,
                       scores_out: Tensor) -> bool:
    """ROCm bbox path: the grouping stage in ONE launch (``ops.coco_prepare``: per image, every detection / ground
    truth ranks itself against the image's (category, score) keys in LDS and writes itself into matcher order, with
    the group starts / counts and the non-ignored ground-truth histogram), then the matcher, ONE (category, score)
    sort and the accumulation kernel.  The same arrays as the ATen grouping below, but ~35 launches instead of ~160
    (compute() was host-bound on them).  False (nothing written) where it does not apply: fp64 scores, images of more
    than ``PREP_MAX_PER_IMAGE`` annotations, non-integer labels / crowds."""
    dev = classes.device
    n_img = len(d_sizes)
    biggest = max(max(d_sizes, default=0), max(g_sizes, default=0))
    if n_img == 0 or biggest > PREP_MAX_PER_IMAGE:
        return False
    d_lab = cat_states(det_labels, dev).reshape(-1)
    g_lab = cat_states(gt_labels, dev).reshape(-1)
    d_score = cat_states(det_scores, dev).reshape(-1)
    g_crowd = cat_states(gt_crowds, dev).reshape(-1)
    g_area = cat_states(gt_areas, dev).reshape(-1)
    d_box = cat_states(det_boxes, dev, (4,))
    g_box = cat_states(gt_boxes, dev, (4,))
    ints, floats = (torch.int64, torch.int32, torch.int16, torch.uint8, torch.bool), \
        (torch.float32, torch.float64, torch.float16, torch.bfloat16)
    if g_area.dtype in ints:  # (no "area" key: the zero defaults carry the labels' dtype)
        g_area = g_area.to(torch.float64)
    if d_score.dtype not in floats[:1] + floats[2:] or any(t.dtype not in ints for t in (d_lab, g_lab, g_crowd)) or \
            any(t.dtype not in floats for t in (d_box, g_box, g_area)):
        return False
    off = [0, *accumulate(d_sizes), 0, *accumulate(g_sizes)]
    K, A = classes.numel(), areas.shape[0]
    G = n_img * K
    (tables, d_box_s, d_area_s, rank_v, cls_k, score_k, key2, g_box_s, g_area_s,
     g_crowd_s) = ops.coco_prepare(classes, _to_device_async(off, dev), d_lab.contiguous(), d_score.contiguous(),
                                   d_box.contiguous(), g_lab.contiguous(), g_box.contiguous(), g_crowd.contiguous(),
                                   g_area.contiguous(), areas.reshape(-1), n_img, int(max_dets[-1]), biggest)
    dt_match, dt_ig = ops.coco_match(d_box_s, d_area_s, g_box_s, g_area_s, g_crowd_s, tables[:G], tables[G:2 * G],
                                     tables[2 * G:3 * G], tables[3 * G:4 * G], areas.reshape(-1), t_thr, None, None)
    npig = tables[4 * G:].reshape(A, K).to(torch.float64)
    # (3) accumulate: detections of each category in score order (ties: image, then rank -- the prepared order);
    # categories not on the K axis carry index K and sort last
    o = torch.sort(key2, stable=True).indices
    # (where the accumulation kernel does not apply -- T * A > 63, more than 8 max-dets values, no detections -- the
    # caller's ATen path runs from the start)
    return ops.coco_accumulate_sorted(dt_match, dt_ig, o, rank_v, score_k, cls_k, npig, r_thr, max_dets, precision,
                                      recall, scores_out)


def _masked_mean(s: Tensor) -> Tensor:
    valid = s > -1
    cnt = valid.sum()
    return torch.where(cnt > 0, (s * valid).sum() / cnt.clamp(min=1), torch.tensor(-1.0, dtype=s.dtype,
                                                                                 device=s.device))


def _masked_sums(ev: Dict[str, Tensor]) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Sums and counts of the defined (> -1) entries: precision over (R, K) -> ``[T, A, M]``, recall over K ->
    ``[T, A, M]`` -- every summary number is a ratio of a few of these (four reductions instead of ~50 launches of
    per-number masked means)."""
    prec, rec = ev["precision"], ev["recall"]
    pv, rv = prec > -1, rec > -1
    return (torch.where(pv, prec, 0.0).sum((1, 2)), pv.sum((1, 2)), torch.where(rv, rec, 0.0).sum(1), rv.sum(1))


def _ratio(num: float, cnt: float) -> float:
    return num / cnt if cnt > 0 else -1.0


def coco_summarize(ev: Dict[str, Tensor], iou_thresholds: Sequence[float], max_dets: Sequence[int],
                   map_max_det: Optional[int] = None, host: Optional[Tuple] = None) -> Tensor:
    """The 12 COCO summary numbers (``COCOeval.summarize``) as a float64 CPU tensor.

    ``map_max_det=100`` reproduces pycocotools' ``summarize``, whose first number (mAP) is taken at a hard-coded 100
    detections -- -1 when 100 is not among ``max_dets`` (the reference's ``backend="pycocotools"``,
    ``T/unittests/detection/test_map.py:826-856``); ``None`` uses the largest threshold (faster-coco-eval).
    The masked sums of :func:`_masked_sums` cross to the host once (``host``: already fetched ones); each number is
    (sum of the selected sums) / (sum of the selected counts), the mean over the defined entries pycocotools takes.
    """
    sp, cp, sr, cr = host if host is not None else (t.double().cpu() for t in _masked_sums(ev))
    thr = list(iou_thresholds)
    last = len(max_dets) - 1

    def ap(iou=None, area=0, m=last):
        ts = [i for i, t in enumerate(thr) if t == iou] if iou is not None else list(range(len(thr)))
        return _ratio(float(sp[ts, area, m].sum()), float(cp[ts, area, m].sum()))

    def ar(area=0, m=last):
        return _ratio(float(sr[:, area, m].sum()), float(cr[:, area, m].sum()))

    first = ap() if map_max_det is None else (
        ap(m=list(max_dets).index(map_max_det)) if map_max_det in max_dets else -1.0)
    stats = [first, ap(0.5), ap(0.75), ap(area=1), ap(area=2), ap(area=3), ar(m=0), ar(m=1), ar(m=2),
             ar(area=1), ar(area=2), ar(area=3)]
    return torch.tensor(stats, dtype=torch.float64)


def per_class_stats(ev: Dict[str, Tensor], max_dets: Optional[Sequence[int]] = None,
                    map_max_det: Optional[int] = None) -> Tuple[Tensor, Tensor]:
    """Per-category mAP (all areas) and mAR at the last max-dets, -1 where undefined; mAP at ``map_max_det``
    detections when given (pycocotools' per-class ``stats[0]``, -1 without such a threshold)."""
    m_ap = -1
    if map_max_det is not None and max_dets is not None:
        m_ap = list(max_dets).index(map_max_det) if map_max_det in max_dets else None
    rec = ev["recall"][..., 0, -1]  # [T, K]
    rv = rec > -1
    r_cnt = rv.sum(0)
    mr = torch.where(r_cnt > 0, torch.where(rv, rec, 0.0).sum(0) / r_cnt.clamp(min=1),
                     torch.full_like(r_cnt, -1.0, dtype=rec.dtype))
    if m_ap is None:
        return torch.full_like(mr, -1.0), mr
    prec = ev["precision"][..., 0, m_ap]  # [T, R, K]
    pv = prec > -1
    p_cnt = pv.sum((0, 1))
    mp = torch.where(p_cnt > 0, torch.where(pv, prec, 0.0).sum((0, 1)) / p_cnt.clamp(min=1),
                     torch.full_like(p_cnt, -1.0, dtype=prec.dtype))
    return mp, mr


def _summary_kernel(ev: Dict[str, Tensor], max_dets: Sequence[int], map_max_det: Optional[int],
                    class_ev: Optional[Dict[str, Tensor]]) -> Optional[Tuple[Tuple[Tensor, ...], Tensor, Tensor]]:
    """ROCm: the masked sums and the per-class numbers from ONE summary launch and one host transfer."""
    prec, rec = ev["precision"], ev["recall"]
    cev = class_ev if class_ev is not None else ev
    m_ap = len(max_dets) - 1
    if map_max_det is not None:
        m_ap = list(max_dets).index(map_max_det) if map_max_det in max_dets else -1
    vec = ops.coco_summary(prec, rec, cev["precision"], cev["recall"], m_ap)
    if vec is None:
        return None
    T, _, K, A, M = prec.shape
    v = vec.cpu()
    tam, tk, nb = T * A * M, T * K, (K + 3) // 4
    sp, cp = (v[i * nb * tam:(i + 1) * nb * tam].reshape(T, nb, A, M).sum(1) for i in range(2))
    base = 2 * nb * tam
    sr, cr = (v[base + i * tam:base + (i + 1) * tam].reshape(T, A, M) for i in range(2))
    base += 2 * tam
    mps, mpc, mrs, mrc = (v[base + i * tk:base + (i + 1) * tk].reshape(T, K).sum(0) for i in range(4))
    mp = torch.where(mpc > 0, mps / mpc.clamp(min=1), torch.full_like(mps, -1.0))
    if m_ap < 0:
        mp = torch.full_like(mps, -1.0)
    mr = torch.where(mrc > 0, mrs / mrc.clamp(min=1), torch.full_like(mrs, -1.0))
    return (sp, cp, sr, cr), mp, mr


def summarize_all(ev: Dict[str, Tensor], iou_thresholds: Sequence[float], max_dets: Sequence[int],
                  map_max_det: Optional[int] = None, class_ev: Optional[Dict[str, Tensor]] = None
                  ) -> Tuple[Tensor, Optional[Tensor], Optional[Tensor]]:
    """The summary numbers and (``class_ev`` given) the per-class mAP / mAR with ONE device->host transfer."""
    fused = _summary_kernel(ev, max_dets, map_max_det, class_ev)
    if fused is not None:
        host, mp, mr = fused
        stats = coco_summarize(ev, iou_thresholds, max_dets, map_max_det, host=host)
        return (stats, None, None) if class_ev is None else (stats, mp, mr)
    parts = list(_masked_sums(ev))
    if class_ev is not None:
        parts += list(per_class_stats(class_ev, max_dets, map_max_det))
    sizes = [p.numel() for p in parts]
    shapes = [p.shape for p in parts]
    flat = torch.cat([p.reshape(-1).double() for p in parts]).cpu()
    host = [x.reshape(sh) for x, sh in zip(torch.split(flat, sizes), shapes)]
    stats = coco_summarize(ev, iou_thresholds, max_dets, map_max_det, host=tuple(host[:4]))
    if class_ev is None:
        return stats, None, None
    return stats, host[4], host[5]


def _rle_iou_blocks(det_rle: Tuple[Tensor, Tensor], gt_rle: Tuple[Tensor, Tensor], crowd: Tensor, d_of: Tensor,
                    g_of: Tensor, grp_s: Tensor, rank: Tensor, max_det: int, det_cnt: Tensor, gt_start: Tensor,
                    gt_cnt: Tensor, n_groups: int) -> Tuple[Tensor, Tensor]:
    """Per-group ``[det, gt]`` mask-IoU blocks laid out for ``coco_match``, from the run-length encoded masks.

    Every (detection, ground truth) pair of a group is one entry of a flat pair list -- block of group ``g`` at
    ``off[g]``, row ``k`` = ``k``-th score-ordered detection, ``gt_cnt[g]`` columns in ground-truth order -- and
    ``ops.rle_iou`` evaluates them all in one launch (crowd ground truths: intersection over detection area).
    ``d_of`` / ``g_of`` map sorted detections / ground truths to their descriptor rows; ``crowd`` is per descriptor row.
    Detections of the sentinel group ``n_groups`` or ranked past ``max_det`` get no block rows.
    """
    dev = grp_s.device
    live = (grp_s < n_groups) & (rank < max_det)
    grp_c = grp_s.clamp(max=n_groups - 1)
    reps = torch.where(live, gt_cnt[grp_c], 0)
    block_rows = torch.repeat_interleave(torch.arange(grp_s.numel(), device=dev), reps)
    col = torch.arange(block_rows.numel(), device=dev) - torch.repeat_interleave(torch.cumsum(reps, 0) - reps, reps)
    pd = d_of[block_rows].contiguous()
    pg = g_of[gt_start[grp_c[block_rows]] + col].contiguous()
    vals = ops.rle_iou(det_rle[0], det_rle[1], gt_rle[0], gt_rle[1], pd, pg, crowd.contiguous())
    sizes = det_cnt * gt_cnt
    return vals.contiguous(), (torch.cumsum(sizes, 0) - sizes).contiguous()
