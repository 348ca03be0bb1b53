"""Plain-Python COCO bbox evaluation oracle (evaluate / accumulate / summarize), written from the COCO protocol.

Used only by the tests to pin the device implementation; loops over images, categories, areas and thresholds in the
obvious way, no vectorisation tricks.
"""
import numpy as np

AREAS = [(0, 1e10), (0, 32**2), (32**2, 96**2), (96**2, 1e10)]


def _iou(d, g, crowd):
    w = min(d[0] + d[2], g[0] + g[2]) - max(d[0], g[0])
    h = min(d[1] + d[3], g[1] + g[3]) - max(d[1], g[1])
    if w <= 0 or h <= 0:
        return 0.0
    inter = w * h
    u = d[2] * d[3] if crowd else d[2] * d[3] + g[2] * g[3] - inter
    return inter / u


def coco_eval(dets, gts, cats, iou_thrs, rec_thrs, max_dets, iou_fn=None, area_fn=None):
    """dets: per image list of (box_xywh, score, cat); gts: per image list of (box_xywh, cat, crowd, area).

    ``iou_fn(d_geom, g_geom, crowd)`` / ``area_fn(d_geom)`` replace the box IoU / area (e.g. dense-mask IoU for segm,
    with the geometry slot holding a numpy mask)."""
    iou_fn = iou_fn or _iou
    area_fn = area_fn or (lambda b: b[2] * b[3])
    T, R, K, A, M = len(iou_thrs), len(rec_thrs), len(cats), len(AREAS), len(max_dets)
    evals = {}
    for img in range(len(dets)):
        for k, c in enumerate(cats):
            dt = [d for d in dets[img] if d[2] == c]
            gt = [g for g in gts[img] if g[1] == c]
            if not dt and not gt:
                continue
            order = sorted(range(len(dt)), key=lambda i: -dt[i][1])[: max_dets[-1]]
            dt = [dt[i] for i in order]
            for a, (lo, hi) in enumerate(AREAS):
                gig = [1 if (g[2] or g[3] < lo or g[3] > hi) else 0 for g in gt]
                gorder = sorted(range(len(gt)), key=lambda i: gig[i])
                gs = [gt[i] for i in gorder]
                gi = [gig[i] for i in gorder]
                dtm = np.zeros((T, len(dt)))
                dtig = np.zeros((T, len(dt)))
                for t, thr in enumerate(iou_thrs):
                    gtm = [0] * len(gs)
                    for di, d in enumerate(dt):
                        best, m = min(thr, 1 - 1e-10), -1
                        for j, g in enumerate(gs):
                            if gtm[j] and not g[2]:
                                continue
                            if m > -1 and gi[m] == 0 and gi[j] == 1:
                                break
                            v = iou_fn(d[0], g[0], g[2])
                            if v < best:
                                continue
                            best, m = v, j
                        if m == -1:
                            continue
                        dtig[t, di] = gi[m]
                        dtm[t, di] = 1
                        gtm[m] = 1
                for di, d in enumerate(dt):
                    area = area_fn(d[0])
                    if area < lo or area > hi:
                        dtig[:, di] = np.where(dtm[:, di] == 0, 1, dtig[:, di])
                evals[(img, k, a)] = (np.array([d[1] for d in dt]), dtm, dtig, np.array(gi))
    precision = -np.ones((T, R, K, A, M))
    recall = -np.ones((T, K, A, M))
    for k in range(K):
        for a in range(A):
            for m, md in enumerate(max_dets):
                E = [evals[(img, k, a)] for img in range(len(dets)) if (img, k, a) in evals]
                if not E:
                    continue
                scores = np.concatenate([e[0][:md] for e in E])
                inds = np.argsort(-scores, kind="mergesort")
                dtm = np.concatenate([e[1][:, :md] for e in E], axis=1)[:, inds]
                dtig = np.concatenate([e[2][:, :md] for e in E], axis=1)[:, inds]
                gig = np.concatenate([e[3] for e in E])
                npig = np.count_nonzero(gig == 0)
                if npig == 0:
                    continue
                tps = np.logical_and(dtm, np.logical_not(dtig))
                fps = np.logical_and(np.logical_not(dtm), np.logical_not(dtig))
                tp_sum = np.cumsum(tps, axis=1).astype(float)
                fp_sum = np.cumsum(fps, axis=1).astype(float)
                for t in range(T):
                    tp, fp = tp_sum[t], fp_sum[t]
                    nd = len(tp)
                    rc = tp / npig
                    pr = list(tp / (fp + tp + np.spacing(1)))
                    recall[t, k, a, m] = rc[-1] if nd else 0
                    for i in range(nd - 1, 0, -1):
                        if pr[i] > pr[i - 1]:
                            pr[i - 1] = pr[i]
                    q = np.zeros(R)
                    idx = np.searchsorted(rc, rec_thrs, side="left")
                    for ri, pi in enumerate(idx):
                        if pi < nd:
                            q[ri] = pr[pi]
                    precision[t, :, k, a, m] = q
    return precision, recall


def summarize(precision, recall, iou_thrs, max_dets):
    def mean(s):
        s = s[s > -1]
        return -1.0 if s.size == 0 else float(np.mean(s))

    def ap(iou=None, a=0, m=len(max_dets) - 1):
        s = precision[..., a, m]
        if iou is not None:
            s = s[[i for i, t in enumerate(iou_thrs) if t == iou]]
        return mean(s)

    def ar(a=0, m=len(max_dets) - 1):
        return mean(recall[..., a, m])

    return [ap(), ap(0.5), ap(0.75), ap(a=1), ap(a=2), ap(a=3), ar(m=0), ar(m=1), ar(m=2), ar(a=1), ar(a=2),
            ar(a=3)]
