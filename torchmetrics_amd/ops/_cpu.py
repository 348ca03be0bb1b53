"""CPU implementations of the ``torch.ops.tm_amd`` contracts (ATen ops, eager validation).

Same inputs/outputs as the HIP kernels in ``csrc/``; invalid values raise immediately (no device flag on the host).
"""
from typing import Optional

import torch
from torch import Tensor

from torchmetrics_amd.utils import validation as V


def _set(flag: Tensor, code: int) -> None:
    """Record a validation failure exactly like the kernels do (the caller decides when to raise)."""
    if flag is not None:
        flag.bitwise_or_(code)


def mc_update(
    preds: Tensor,
    target: Tensor,
    out: Tensor,
    flag: Tensor,
    num_classes: int,
    ignore_index: Optional[int],
    mode: int,
    samplewise: bool,
) -> None:
    C = int(num_classes)
    N = target.shape[0] if target.ndim else 1
    if target.numel() == 0:
        return
    target = target.reshape(N, -1).long()
    X = target.shape[1]
    if preds.is_floating_point():
        labels = preds.reshape(N, C, X).argmax(dim=1).unsqueeze(1)  # [N, 1, X]
    else:
        labels = preds.reshape(N, -1, X).long()  # [N, K, X]
    K = labels.shape[1]
    valid = torch.ones_like(target, dtype=torch.bool)
    if ignore_index is not None:
        valid &= target != ignore_index
    bad_t = valid & ((target < 0) | (target >= C))
    if bool(bad_t.any()):
        _set(flag, V.TARGET_OUT_OF_RANGE)
        valid &= ~bad_t
    bad_p = ((labels < 0) | (labels >= C)).any(dim=1) & valid
    if bool(bad_p.any()):
        _set(flag, V.PREDS_OUT_OF_RANGE)
        valid &= ~bad_p
    if mode == 0:
        t = target[valid]
        p = labels[:, 0, :][valid]
        out.view(-1).add_(torch.bincount(t * C + p, minlength=C * C))
        return
    G = N if samplewise else 1
    ws = out.view(G, 3 * C + 1)
    if K == 1 and not samplewise:
        t = target[valid]
        p = labels[:, 0, :][valid]
        cm = torch.bincount(t * C + p, minlength=C * C).view(C, C)
        tp = cm.diag()
        ws[0, :C] += tp
        ws[0, C : 2 * C] += cm.sum(0) - tp
        ws[0, 2 * C : 3 * C] += cm.sum(1) - tp
        return
    onehot_t = torch.nn.functional.one_hot(target.clamp(0, C - 1), C) * valid.unsqueeze(-1)  # [N, X, C]
    pred_set = torch.zeros(N, X, C, dtype=torch.long)
    pred_set.scatter_(2, labels.clamp(0, C - 1).permute(0, 2, 1), 1)
    pred_set = pred_set * valid.unsqueeze(-1)
    tp = (onehot_t * pred_set).sum(1)  # [N, C]
    fn = (onehot_t * (1 - pred_set)).sum(1)
    fp = ((1 - onehot_t) * pred_set).sum(1)
    if not samplewise:
        tp, fp, fn = tp.sum(0, keepdim=True), fp.sum(0, keepdim=True), fn.sum(0, keepdim=True)
    ws[:, :C] += tp
    ws[:, C : 2 * C] += fp
    ws[:, 2 * C : 3 * C] += fn


def mc_stats_finalize(ws: Tensor, num_classes: int, micro: bool, accumulate: bool, tp: Tensor, fp: Tensor,
                      tn: Tensor, fn: Tensor) -> None:
    C = int(num_classes)
    G = ws.numel() // (3 * C + 1)
    w = ws.view(G, 3 * C + 1)
    a, b, d = w[:, :C], w[:, C : 2 * C], w[:, 2 * C : 3 * C]
    # every counted row added one to tp[t] or fn[t]: the row count of a group is sum(tp + fn) (the last slot of each
    # group is unused, as in csrc/classification/stat_scores.hip)
    cnt = (a + d).sum(1, keepdim=True)
    if micro:
        a, b, d = a.sum(1), b.sum(1), d.sum(1)
        e = C * cnt[:, 0] - a - b - d
    else:
        e = cnt - a - b - d
    for dst, src in ((tp, a), (fp, b), (fn, d), (tn, e)):
        src = src.reshape(dst.shape)
        if accumulate:
            dst += src
        else:
            dst.copy_(src)
    w.zero_()


def bin_update(preds: Tensor, target: Tensor, ws: Tensor, flag: Tensor, not_prob: Tensor, num_labels: int,
               threshold: float, ignore_index: Optional[int], samplewise: bool, prob_check_all: bool = True) -> None:
    if preds.numel() == 0:
        return
    N = preds.shape[0]
    L = int(num_labels)
    p = preds.reshape(N, L, -1)
    t = target.reshape(N, L, -1).long()
    valid = torch.ones_like(t, dtype=torch.bool)
    if ignore_index is not None:
        valid &= t != ignore_index
    bad_t = valid & (t != 0) & (t != 1)
    if bool(bad_t.any()):
        _set(flag, V.TARGET_NOT_BINARY)
        valid &= ~bad_t
    if p.is_floating_point():
        in_range = (p >= 0) & (p <= 1)
        if not prob_check_all and ignore_index is not None:
            in_range = in_range | (t == ignore_index)
        if not bool(in_range.all()):
            not_prob.fill_(1)
        thr = torch.tensor(threshold, dtype=p.dtype)
        pa = p > thr
        pb = p.float().sigmoid().to(p.dtype) > thr
    else:
        bad_p = (p != 0) & (p != 1)
        if bool(bad_p.any()):
            _set(flag, V.PREDS_NOT_BINARY)
            valid &= ~bad_p
        pa = pb = p == 1
    tt = (t == 1) & valid
    tf = (t == 0) & valid
    sum_dims = (2,) if samplewise else (0, 2)
    cols = [
        (tt & pa).sum(sum_dims), (tf & pa).sum(sum_dims), (tt & ~pa).sum(sum_dims),
        (tt & pb).sum(sum_dims), (tf & pb).sum(sum_dims), (tt & ~pb).sum(sum_dims),
        valid.sum(sum_dims),
    ]
    ws.view(-1, 7).add_(torch.stack([c.reshape(-1) for c in cols], dim=1))


def bin_stats_finalize(ws: Tensor, not_prob: Tensor, accumulate: bool, tp: Tensor, fp: Tensor, tn: Tensor,
                       fn: Tensor) -> None:
    w = ws.view(-1, 7)
    off = 3 if int(not_prob.reshape(-1)[0].item()) else 0
    a, b, d = w[:, off], w[:, off + 1], w[:, off + 2]
    e = w[:, 6] - a - b - d
    for dst, src in ((tp, a), (fp, b), (fn, d), (tn, e)):
        src = src.reshape(dst.shape)
        if accumulate:
            dst += src
        else:
            dst.copy_(src)
    w.zero_()
    not_prob.zero_()


def bin_confmat_finalize(ws: Tensor, not_prob: Tensor, confmat: Tensor) -> None:
    w = ws.view(-1, 7)
    off = 3 if int(not_prob.reshape(-1)[0].item()) else 0
    tp, fp, fn = w[:, off], w[:, off + 1], w[:, off + 2]
    tn = w[:, 6] - tp - fp - fn
    confmat.view(-1, 4).add_(torch.stack([tn, fp, fn, tp], dim=1))
    w.zero_()
    not_prob.zero_()


def moments_update(preds, target, num_outputs, mask, eps, power, shift_p, shift_t, dests, dest_ids, want_sums,
                   fold=0):
    k = int(num_outputs)
    p = preds.reshape(-1, k).double()
    t = target.reshape(-1, k).double()
    d = p - t
    ad = d.abs()
    sums = torch.zeros(k, 19, dtype=torch.float64, device=p.device)
    pc = p - (shift_p.double() if shift_p is not None else 0.0)
    tc = t - (shift_t.double() if shift_t is not None else 0.0)
    cols = {
        0: lambda: (d * d).sum(0),
        1: lambda: ad.sum(0),
        2: lambda: pc.sum(0),
        3: lambda: tc.sum(0),
        4: lambda: (pc * pc).sum(0),
        5: lambda: (tc * tc).sum(0),
        6: lambda: (pc * tc).sum(0),
        7: lambda: (ad / t.abs().clamp(min=eps)).sum(0),
        8: lambda: (2 * ad / (p.abs() + t.abs()).clamp(min=eps)).sum(0),
        9: lambda: t.abs().sum(0),
        10: lambda: ((torch.log1p(p) - torch.log1p(t)) ** 2).sum(0),
        11: lambda: (ad + torch.log1p(torch.exp(-2 * ad)) - 0.69314718055994530942).sum(0),
        12: lambda: (ad**power).sum(0),
        13: lambda: torch.full((k,), float(p.shape[0]), dtype=torch.float64, device=p.device),
        14: lambda: p.sum(0),
        15: lambda: t.sum(0),
        16: lambda: (p * p).sum(0),
        17: lambda: (t * t).sum(0),
        18: lambda: (p * t).sum(0),
    }
    for sid, fn in cols.items():
        if mask & (1 << sid) or sid == 13:
            sums[:, sid] = fn()
    if fold == 1:  # Pearson running-moment fold (first 6 dests), same formulation as csrc/regression/moments.hip
        mean_x, mean_y, m2_x, m2_y, c_xy, n0 = dests[:6]
        dests = dests[6:]
        sd, se, sdd, see, sde = (sums[:, i] for i in (2, 3, 4, 5, 6))
        tot = n0.reshape(k).double() + p.shape[0]
        dx, dy = sd / tot, se / tot
        for dst, inc in ((mean_x, dx), (mean_y, dy), (m2_x, sdd - dx * sd), (m2_y, see - dy * se),
                         (c_xy, sde - dx * se)):
            dst += inc.reshape(dst.shape).to(dst.dtype)
        n0 += p.shape[0]
    for dst, sid in zip(dests, dest_ids):
        col = sums[:, sid] if sid < 32 else sums[:, (sid - 32) // 32] - sums[:, (sid - 32) % 32]
        val = col if dst.numel() == k else col[0]
        if dst.dtype == torch.int64:
            val = torch.round(val).long()
        dst += val.reshape(dst.shape).to(dst.dtype)
    return sums if want_sums else None


def feature_moments_update(features: Tensor, feat_sum: Tensor, feat_cov: Tensor) -> None:
    x = features.double()
    feat_sum += x.sum(0)
    feat_cov += x.t().mm(x)


def curve_update(preds: Tensor, target: Tensor, thr_sorted: Tensor, perm: Tensor, state: Tensor, err: Tensor,
                 mode: int, ignore_index: Optional[int], micro: bool) -> None:
    """Bucket every score by ``#{thr <= p}`` (one ``bucketize``), histogram, suffix-sum -> per-threshold confmats."""
    t = thr_sorted.numel()
    if mode == 2:  # multiclass
        c = preds.shape[1]
        keep = torch.ones_like(target, dtype=torch.bool) if ignore_index is None else target != ignore_index
        p, tg = preds[keep], target[keep].long()
        if p.numel() and not torch.all((p >= 0) & (p <= 1)):
            p = p.softmax(1)
        bad = (tg < 0) | (tg >= c)
        if bool(bad.any()):
            _set(err, V.TARGET_OUT_OF_RANGE)
            p, tg = p[~bad], tg[~bad]
        pos = torch.nn.functional.one_hot(tg, c) if tg.numel() else torch.zeros(0, c, dtype=torch.long)
        cols = c
    else:
        if mode == 0:
            p, tg = preds.reshape(-1, 1), target.reshape(-1, 1).long()
            keep = torch.ones_like(tg, dtype=torch.bool) if ignore_index is None else tg != ignore_index
            check = p[keep]
        else:
            p, tg = preds, target.long()
            keep = torch.ones_like(tg, dtype=torch.bool) if ignore_index is None else tg != ignore_index
            check = p
        if check.numel() and not torch.all((check >= 0) & (check <= 1)):
            p = p.sigmoid()
        bad = keep & (tg != 0) & (tg != 1)
        if bool(bad.any()):
            _set(err, V.TARGET_NOT_BINARY)
        keep = keep & ~bad
        pos = tg.clamp(0, 1)
        cols = p.shape[1]
    b = torch.bucketize(p.double(), thr_sorted.to(p.device), right=True)  # #{thr <= p}; NaN -> T (fixed below)
    b = torch.where(torch.isnan(p), torch.zeros_like(b), b)
    col = torch.arange(cols).expand_as(b)
    if mode == 2:
        keep = torch.ones_like(b, dtype=torch.bool)
    if micro:
        col = torch.zeros_like(col)
        cols = 1
    idx = ((b * cols + col) * 2 + pos)[keep]
    hist = torch.bincount(idx, minlength=(t + 1) * cols * 2).reshape(t + 1, cols, 2)
    suffix = hist.flip(0).cumsum(0).flip(0)  # suffix[b] = counts in buckets >= b
    tot = suffix[0]
    above = suffix[1:]  # sorted threshold i: predicted positive <=> bucket >= i + 1
    out = torch.stack([tot[:, 0] - above[:, :, 0], above[:, :, 0], tot[:, 1] - above[:, :, 1], above[:, :, 1]], -1)
    res = torch.empty_like(out)
    res[perm] = out
    state += res.reshape(state.shape)


def ssim2d_partials(x: Tensor, y: Tensor, wh: Tensor, ww: Tensor, c12: Tensor, mode: int) -> Tensor:
    """Valid-window SSIM / UQI sums per plane via one separable depthwise convolution of the 5 moment maps."""
    acc = torch.float64 if x.dtype == torch.float64 else torch.float32
    x, y = x.to(acc).unsqueeze(1), y.to(acc).unsqueeze(1)
    k = (wh.to(acc)[:, None] * ww.to(acc)[None, :])[None, None]
    maps = torch.cat([x, y, x * x, y * y, x * y], 1)  # [P, 5, H, W]
    m = torch.nn.functional.conv2d(maps, k.expand(5, 1, -1, -1), groups=5)
    mx, my, exx, eyy, exy = m.unbind(1)
    mxx, myy, mxy = mx * mx, my * my, mx * my
    sxx, syy, sxy = (exx - mxx).clamp(min=0), (eyy - myy).clamp(min=0), exy - mxy
    c1, c2, eps = (float(v) for v in c12.to(acc).cpu()[:3])
    if mode == 0:
        upper, lower = 2 * sxy + c2, sxx + syy + c2
        val = ((2 * mxy + c1) * upper) / ((mxx + myy + c1) * lower)
        cs = upper / lower
    elif mode == 3:  # spatial correlation coefficient of high-passed planes
        den = sxx.sqrt() * syy.sqrt()
        val = torch.where(den == 0, torch.zeros_like(sxy), sxy / torch.where(den == 0, 1.0, den))
        cs = torch.zeros_like(val)
    elif mode == 2:  # one VIF scale: x reference, y distorted, c1 = sigma_n^2
        stt = sxx
        g = sxy / (sxx + eps)
        sv = syy - g * sxy
        low_t = stt < eps
        g, sv, stt = torch.where(low_t, 0.0, g), torch.where(low_t, syy, sv), torch.where(low_t, 0.0, stt)
        low_p = syy < eps
        g, sv = torch.where(low_p, 0.0, g), torch.where(low_p, 0.0, sv)
        neg = g < 0
        sv, g = torch.where(neg, syy, sv), torch.where(neg, 0.0, g)
        sv = sv.clamp(min=eps)
        val = torch.log10(1.0 + g * g * stt / (sv + c1))
        cs = torch.log10(1.0 + stt / c1)
    else:
        upper, lower = 2 * sxy, sxx + syy
        val = ((2 * mxy) * upper) / ((mxx + myy) * lower + eps)
        cs = torch.zeros_like(val)
    return torch.stack([val.flatten(1).sum(1), cs.flatten(1).sum(1)], -1).unsqueeze(1)


def box_pairwise(a: Tensor, b: Tensor, op: int, aligned: bool) -> Tensor:
    acc = torch.float64 if a.dtype == torch.float64 else torch.float32
    out_dtype = a.dtype if a.is_floating_point() else torch.float32
    a, b = a.to(acc), b.to(acc)
    if aligned:
        pa, pb = a, b
    else:
        pa, pb = a[:, None, :], b[None, :, :]
    area_a = (pa[..., 2] - pa[..., 0]) * (pa[..., 3] - pa[..., 1])
    area_b = (pb[..., 2] - pb[..., 0]) * (pb[..., 3] - pb[..., 1])
    iw = (torch.minimum(pa[..., 2], pb[..., 2]) - torch.maximum(pa[..., 0], pb[..., 0])).clamp(min=0)
    ih = (torch.minimum(pa[..., 3], pb[..., 3]) - torch.maximum(pa[..., 1], pb[..., 1])).clamp(min=0)
    inter = iw * ih
    union = area_a + area_b - inter
    iou = inter / union
    if op == 0:
        return iou.to(out_dtype)
    cw = torch.maximum(pa[..., 2], pb[..., 2]) - torch.minimum(pa[..., 0], pb[..., 0])
    ch = torch.maximum(pa[..., 3], pb[..., 3]) - torch.minimum(pa[..., 1], pb[..., 1])
    if op == 1:
        area_c = cw * ch
        return (iou - (area_c - union) / area_c).to(out_dtype)
    eps = 1e-7
    diag = cw**2 + ch**2 + eps
    dx = (pa[..., 0] + pa[..., 2]) / 2 - (pb[..., 0] + pb[..., 2]) / 2
    dy = (pa[..., 1] + pa[..., 3]) / 2 - (pb[..., 1] + pb[..., 3]) / 2
    diou = iou - (dx**2 + dy**2) / diag
    if op == 2:
        return diou.to(out_dtype)
    wa, ha = pa[..., 2] - pa[..., 0], pa[..., 3] - pa[..., 1]
    wb, hb = pb[..., 2] - pb[..., 0], pb[..., 3] - pb[..., 1]
    v = (4 / (torch.pi**2)) * (torch.atan(wb / hb) - torch.atan(wa / ha)) ** 2
    alpha = v / (1 - iou + v + eps)
    return (diou - alpha * v).to(out_dtype)


def _coco_iou(d, g, crowd):
    w = min(d[0] + d[2], g[0] + g[2]) - max(d[0], g[0])
    if w <= 0:
        return 0.0
    h = min(d[1] + d[3], g[1] + g[3]) - max(d[1], g[1])
    if h <= 0:
        return 0.0
    inter = w * h
    da = d[2] * d[3]
    return inter / (da if crowd else da + g[2] * g[3] - inter)


def coco_match(dbox, darea, gbox, garea, gcrowd, det_start, det_cnt, gt_start, gt_cnt, area_rng, iou_thr,
               iou_pre=None, iou_off=None):
    """Host reference of ``coco_match_kernel`` (same greedy COCO semantics, plain loops)."""
    t_n, a_n, d_n = iou_thr.numel(), area_rng.numel() // 2, dbox.shape[0]
    dt_match = torch.zeros(t_n, a_n, d_n, dtype=torch.uint8)
    dt_ig = torch.zeros(t_n, a_n, d_n, dtype=torch.uint8)
    db, da, gb, ga, gc = dbox.tolist(), darea.tolist(), gbox.tolist(), garea.tolist(), gcrowd.tolist()
    rng = area_rng.reshape(-1, 2).tolist()
    thrs = iou_thr.tolist()
    pre = iou_pre.tolist() if iou_pre is not None else None
    offs = iou_off.tolist() if iou_off is not None else None
    for grp, (d0, dn, g0, gn) in enumerate(zip(det_start.tolist(), det_cnt.tolist(), gt_start.tolist(),
                                              gt_cnt.tolist())):
        if dn == 0:
            continue
        if pre is not None:
            ious = [[pre[offs[grp] + k * gn + j] for j in range(gn)] for k in range(dn)]
        else:
            ious = [[_coco_iou(db[d0 + k], gb[g0 + j], gc[g0 + j] != 0) for j in range(gn)] for k in range(dn)]
        for a, (lo, hi) in enumerate(rng):
            ig = [gc[g0 + j] != 0 or ga[g0 + j] < lo or ga[g0 + j] > hi for j in range(gn)]
            order = [j for j in range(gn) if not ig[j]] + [j for j in range(gn) if ig[j]]
            for t, thr in enumerate(thrs):
                used = [False] * gn
                for k in range(dn):
                    best, m = min(thr, 1 - 1e-10), -1
                    for j in order:
                        if used[j] and not gc[g0 + j]:
                            continue
                        if m > -1 and not ig[m] and ig[j]:
                            break
                        if ious[k][j] < best:
                            continue
                        best, m = ious[k][j], j
                    di = d0 + k
                    if m >= 0:
                        used[m] = True
                        dt_match[t, a, di] = 1
                        dt_ig[t, a, di] = int(ig[m])
                    else:
                        dt_ig[t, a, di] = int(da[di] < lo or da[di] > hi)
    return dt_match, dt_ig


def pairwise_distance(x: Tensor, y: Tensor, metric: int, p: float, zero_diagonal: bool,
                      reduction: Optional[str]) -> Tensor:
    """Difference-form distances in fp64 (no norm-expansion cancellation), cast back to the input dtype."""
    dt = x.dtype if x.is_floating_point() else torch.float32
    pp = 1.0 if metric == 0 else (2.0 if metric == 1 else float(p))  # 2 = Lp, 3 = integer Lp
    dist = torch.cdist(x.double(), y.double(), p=pp, compute_mode="donot_use_mm_for_euclid_dist")
    if zero_diagonal:
        k = min(dist.shape)
        dist[torch.arange(k), torch.arange(k)] = 0
    if reduction == "sum":
        dist = dist.sum(-1)
    elif reduction == "mean":
        dist = dist.mean(-1)
    return dist.to(dt)


def levenshtein(pred, poff, ref, roff, out, ins, dele, sub, use_beam, max_ref_len) -> None:
    """Python DP with the same (optional tercom-beam) semantics as ``csrc/text/levenshtein.hip``."""
    import math

    inf = 1 << 28
    p_all, r_all = pred.tolist(), ref.tolist()
    po, ro = poff.tolist(), roff.tolist()
    for b in range(len(po) - 1):
        p, r = p_all[po[b]:po[b + 1]], r_all[ro[b]:ro[b + 1]]
        plen, rlen = len(p), len(r)
        ratio = rlen / plen if plen else 1.0
        width = math.ceil(ratio / 2 + 25) if ratio / 2 > 25 else 25
        prev = [j * ins for j in range(rlen + 1)]
        for i in range(1, plen + 1):
            lo, hi = 0, rlen + 1
            if use_beam:
                diag = math.floor(i * ratio)
                lo = max(0, diag - width)
                hi = rlen + 1 if i == plen else min(rlen + 1, diag + width)
            cur = [inf] * (rlen + 1)
            tok = p[i - 1]
            for j in range(lo, hi):
                v = prev[j] + dele if prev[j] < inf else inf
                if j > 0:
                    if prev[j - 1] < inf:
                        v = min(v, prev[j - 1] + (0 if r[j - 1] == tok else sub))
                    if cur[j - 1] < inf:
                        v = min(v, cur[j - 1] + ins)
                cur[j] = v
            prev = cur
        out[b] = prev[rlen]


def token_nll(logits: Tensor, target: Tensor, ignore_index: Optional[int]) -> Tensor:
    acc = torch.float64 if logits.dtype == torch.float64 else torch.float32
    t = target.long()
    mask = torch.ones_like(t, dtype=torch.bool) if ignore_index is None else t != ignore_index
    safe = torch.where(mask, t, torch.zeros_like(t))
    if bool(((safe < 0) | (safe >= logits.shape[1])).any()):
        raise IndexError("Perplexity: target index out of range of the vocabulary")
    lp = torch.log_softmax(logits.to(acc), dim=1).gather(1, safe[:, None])[:, 0]
    return torch.where(mask, -lp, torch.zeros_like(lp)).float()


def symmetric_toeplitz(vector: Tensor) -> Tensor:
    """``[..., L] -> [..., L, L]`` with ``T[i, j] = v[|i - j|]``."""
    n = vector.shape[-1]
    idx = torch.arange(n, device=vector.device)
    return vector[..., (idx[:, None] - idx[None, :]).abs()]


def toeplitz_solve(r: Tensor, b: Tensor) -> Tensor:
    return torch.linalg.solve(symmetric_toeplitz(r), b.unsqueeze(-1)).squeeze(-1)


def lpips_layer(f0: Tensor, f1: Tensor, w: Tensor, eps: float) -> Tensor:
    n0 = f0 / (torch.sqrt((f0**2).sum(1, keepdim=True)) + eps)
    n1 = f1 / (torch.sqrt((f1**2).sum(1, keepdim=True)) + eps)
    d = ((n0 - n1) ** 2 * w.reshape(1, -1, 1, 1)).sum(1)
    return d.mean(dim=(-2, -1))


def biquad_cascade(x: Tensor, coefs: Tensor, rep: int, clamp: bool) -> Tensor:
    from scipy.signal import lfilter

    xs = x.numpy()
    n_f = coefs.shape[0]
    rows = []
    for r in range(xs.shape[0] * rep):
        v = xs[r // rep]
        for sec in coefs[r % n_f].numpy():
            v = lfilter(sec[:3], sec[3:], v)
            if clamp:
                v = v.clip(-1.0, 1.0)
        rows.append(v)
    import numpy as np

    return torch.from_numpy(np.stack(rows)) if rows else torch.zeros(0, x.shape[1], dtype=torch.float64)


def nms(boxes: Tensor, scores: Tensor, iou_threshold: float, idxs: Optional[Tensor] = None) -> Tensor:
    n = boxes.shape[0]
    if n == 0:
        return torch.empty(0, dtype=torch.long, device=boxes.device)
    order = torch.sort(scores, descending=True, stable=True).indices
    b = boxes[order].float()
    area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    lt = torch.maximum(b[:, None, :2], b[None, :, :2])
    rb = torch.minimum(b[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    sup = inter / (area[:, None] + area[None, :] - inter) > iou_threshold
    if idxs is not None:
        c = idxs[order]
        sup &= c[:, None] == c[None, :]
    sup = torch.triu(sup, diagonal=1).cpu()
    removed = torch.zeros(n, dtype=torch.bool)
    keep = []
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        removed |= sup[i]
    return order[torch.tensor(keep, dtype=torch.long, device=boxes.device)]


# ------------------------------------------------------------------------------------- sorted curves (clf_curve)
def clf_curve(scores: Tensor, target: Tensor, weights: Optional[Tensor], S: int, M: int, seg_stride: int,
              elem_stride: int, tmode: int, pos_label: int, ignore_index: Optional[int], emit: int):
    """Host implementation of ``csrc/sort/clf_curve.hip`` (same outputs, same layout).

    Returns ``[stats [S, 8] (P, N, area, ap, coverage, 0, nruns, 0), fps, tps, thr ([S, M], compacted per segment at
    the run index; ``None`` unless ``emit & 1``), ranks ([S * M] average 1-based ranks by flat id; ``emit & 2``)]``.
    """
    f64 = torch.float64
    sc = scores.as_strided((S, M), (seg_stride, elem_stride), scores.storage_offset()).to(f64)
    if tmode == 2:
        tg = target.as_strided((S, M), (seg_stride, elem_stride), target.storage_offset())
    else:
        tg = target.reshape(1, M).expand(S, M)
    tg = tg.long()
    valid = tg != ignore_index if ignore_index is not None else torch.ones_like(tg, dtype=torch.bool)
    if tmode == 1:
        pos = tg == torch.arange(S).unsqueeze(1)
    else:
        pos = tg == pos_label
    pos = pos & valid
    w = weights.to(f64).reshape(1, M).expand(S, M) if weights is not None else torch.ones(S, M, dtype=f64)
    pw = torch.where(pos, w, torch.zeros_like(w))
    nw = torch.where(valid & ~pos, w, torch.zeros_like(w))
    # order: valid first, then descending score (NaN first), stable
    canon = torch.where(torch.isnan(sc), torch.full_like(sc, float("inf")), sc)
    _, o1 = torch.sort(canon, dim=1, descending=True, stable=True)
    _, o2 = torch.sort((~valid).gather(1, o1).to(torch.int8), dim=1, stable=True)
    order = o1.gather(1, o2)
    s_sc, s_val = sc.gather(1, order), valid.gather(1, order)
    s_pw, s_nw = pw.gather(1, order), nw.gather(1, order)
    key = torch.where(torch.isnan(s_sc), torch.full_like(s_sc, float("inf")), s_sc)
    nan = torch.isnan(s_sc)
    same_prev = torch.zeros_like(s_val)
    same_prev[:, 1:] = (key[:, 1:] == key[:, :-1]) & (nan[:, 1:] == nan[:, :-1])
    start = s_val & ~same_prev
    nxt_same = torch.zeros_like(s_val)
    nxt_same[:, :-1] = same_prev[:, 1:] & s_val[:, 1:]
    end = s_val & ~nxt_same
    tps, fps = s_pw.cumsum(1), s_nw.cumsum(1)
    idx = torch.arange(M).unsqueeze(0).expand(S, M)
    sidx = torch.where(start, idx, torch.full_like(idx, -1)).cummax(1).values.clamp(min=0)
    tp_b = tps.gather(1, sidx) - s_pw.gather(1, sidx)
    fp_b = fps.gather(1, sidx) - s_nw.gather(1, sidx)
    pos_r, neg_r = tps - tp_b, fps - fp_b
    zero = torch.zeros_like(tps)
    area = torch.where(end, neg_r * (tp_b + 0.5 * pos_r), zero).sum(1)
    tot = tps + fps
    ap = torch.where(end & (tot > 0), pos_r * tps / torch.where(tot > 0, tot, torch.ones_like(tot)), zero).sum(1)
    cov = torch.where(end & (pos_r > 0), tot, zero).amax(1) if M else zero.sum(1)
    stats = torch.zeros(S, 8, dtype=f64)
    stats[:, 0], stats[:, 1], stats[:, 2], stats[:, 3], stats[:, 4] = pw.sum(1), nw.sum(1), area, ap, cov
    stats[:, 6] = start.sum(1).to(f64)
    out = [stats, None, None, None, None]
    rid = start.long().cumsum(1) - 1
    if emit & 1:
        c_fps, c_tps, c_thr = (torch.zeros(S, M, dtype=f64) for _ in range(3))
        seg = torch.arange(S).unsqueeze(1).expand(S, M)
        c_fps[seg[end], rid[end]] = fps[end]
        c_tps[seg[end], rid[end]] = tps[end]
        c_thr[seg[end], rid[end]] = s_sc[end]
        out[1:4] = [c_fps, c_tps, c_thr]
    if emit & 2:
        eidx = torch.where(end, idx, torch.full_like(idx, M)).flip(1).cummin(1).values.flip(1)
        rank = 0.5 * (sidx.to(f64) + eidx.to(f64)) + 1.0
        flat = torch.arange(S).unsqueeze(1) * M + order
        ranks = torch.empty(S * M, dtype=f64)
        ranks[flat.reshape(-1)] = rank.reshape(-1)
        out[4] = ranks
    return out


RETRIEVAL_KINDS = ("map", "mrr", "precision", "recall", "fall_out", "hit_rate", "r_precision", "ndcg", "auroc")


def retrieval_metric(preds: Tensor, target: Tensor, indexes: Tensor, kind: int, top_k: int, adaptive_k: bool):
    """Host implementation of ``csrc/sort/retrieval.hip``: per-query values, empty flags, query count."""
    from torchmetrics_amd.functional.retrieval import metrics as R
    from torchmetrics_amd.functional.retrieval._segments import Segments

    seg = Segments(preds, target, indexes)
    k = None if top_k <= 0 else int(top_k)
    name = RETRIEVAL_KINDS[kind]
    fn = {
        "map": lambda: R._seg_average_precision(seg, k),
        "mrr": lambda: R._seg_reciprocal_rank(seg, k),
        "precision": lambda: R._seg_precision(seg, k, adaptive_k),
        "recall": lambda: R._seg_recall(seg, k),
        "fall_out": lambda: R._seg_fall_out(seg, k),
        "hit_rate": lambda: R._seg_hit_rate(seg, k),
        "r_precision": lambda: R._seg_r_precision(seg),
        "ndcg": lambda: R._seg_ndcg(seg, k),
        "auroc": lambda: R._seg_auroc(seg, k),
    }[name]
    n = preds.numel()
    vals = torch.zeros(n, dtype=torch.float64)
    empty = torch.zeros(n, dtype=torch.uint8)
    g = seg.num_groups
    vals[:g] = torch.nan_to_num(fn().to(torch.float64), nan=0.0)
    pos = (seg.target > 0).to(torch.long)
    tot = seg.seg_sum(1 - pos) if name == "fall_out" else seg.seg_sum(pos)
    empty[:g] = (tot == 0).to(torch.uint8)
    return [vals, empty, torch.tensor([g], dtype=torch.int32)]


def retrieval_pr_curve(preds: Tensor, target: Tensor, indexes: Tensor, max_k: int, adaptive_k: bool):
    """Host implementation of ``retrieval_pr_curve`` in ``csrc/sort/retrieval.hip``."""
    from torchmetrics_amd.functional.retrieval import metrics as R
    from torchmetrics_amd.functional.retrieval._segments import Segments

    seg = Segments(preds, target, indexes)
    k = int(max_k) if max_k > 0 else int(seg.size.max()) if seg.num_groups else 0
    empty = (seg.seg_sum((seg.target > 0).to(torch.long)) == 0)
    if seg.num_groups == 0 or k == 0:
        z = torch.zeros(seg.num_groups, k, dtype=torch.float32)
        return [z, z.clone(), empty.to(torch.uint8)]
    p, r, _ = R._seg_pr_curve(seg, k, adaptive_k)
    e = empty.unsqueeze(1)
    return [torch.where(e, torch.zeros_like(p), p), torch.where(e, torch.zeros_like(r), r), empty.to(torch.uint8)]


def paired_cosine(a: Tensor, b: Tensor, scale: float) -> Tensor:
    """Host implementation of ``paired_cosine`` (``csrc/multimodal/clip.hip``)."""
    acc = torch.float64 if a.dtype == torch.float64 else torch.float32
    a, b = a.to(acc), b.to(acc)
    return (scale * (a * b).sum(-1) / (a.norm(dim=-1) * b.norm(dim=-1))).to(torch.float32)


def prompt_pair_prob(img: Tensor, anchors: Tensor, scale: float) -> Tensor:
    """Host implementation of ``prompt_pair_prob`` (``csrc/multimodal/clip.hip``)."""
    acc = torch.float64 if img.dtype == torch.float64 else torch.float32
    logits = scale * img.to(acc) @ anchors.to(acc).t()
    return logits.reshape(logits.shape[0], -1, 2).softmax(-1)[:, :, 0].to(torch.float32)


def kendall_stats(x: Tensor, y: Tensor) -> Tensor:
    """Host implementation of ``csrc/sort/kendall.hip`` (Knight's method in batched torch ops)."""
    from torchmetrics_amd.functional.regression import correlation as C

    _, disc = C._pair_counts(x, y)
    tx, tx1, tx2 = C._tie_stats(x)
    ty, ty1, ty2 = C._tie_stats(y)
    n, k = x.shape
    txy = torch.zeros(k, dtype=torch.float64)
    ux = torch.zeros(k, dtype=torch.float64)
    uy = torch.zeros(k, dtype=torch.float64)
    for c in range(k):
        _, cnt = torch.unique(torch.stack([x[:, c], y[:, c]], 1), dim=0, return_counts=True)
        cnt = cnt.double()
        txy[c] = (cnt * (cnt - 1) / 2).sum()
        ux[c] = float(torch.unique(x[:, c]).numel())
        uy[c] = float(torch.unique(y[:, c]).numel())
    return torch.stack([disc.double(), tx, tx1, tx2, ty, ty1, ty2, txy, ux, uy], 1)


_GEMM_TILE = 128


def gemm_nt(x: Tensor, y: Tensor, kind: int, aux_x, aux_y, scale: float, coef: float, degree: int,
            zero_diagonal: bool, sqrt_out: bool) -> Tensor:
    """Host implementation of ``csrc/pairwise/gemm_nt.hip`` (same outputs / partial layouts)."""
    xf, yf = x.float(), y.float()
    batched = xf.dim() == 3
    if not batched:
        xf, yf = xf.unsqueeze(0), yf.unsqueeze(0)
        aux_x = None if aux_x is None else aux_x.reshape(1, -1)
        aux_y = None if aux_y is None else aux_y.reshape(1, -1)
    b, n, m = xf.shape[0], xf.shape[1], yf.shape[1]
    dot = torch.bmm(xf, yf.transpose(1, 2))
    eye = torch.eye(n, m, dtype=torch.bool).unsqueeze(0)
    if kind in (0, 1, 2):
        if kind == 0:
            out = dot * scale
        elif kind == 2:
            out = dot * aux_x.reshape(b, n, 1).float() * aux_y.reshape(b, 1, m).float() * scale
        else:
            d2 = aux_x.reshape(b, n, 1).float() + aux_y.reshape(b, 1, m).float() - 2 * dot
            exact = torch.cdist(xf.double(), yf.double()).pow(2).float()
            d2 = torch.where(d2 < (aux_x.reshape(b, n, 1) + aux_y.reshape(b, 1, m)).float() / 128, exact, d2)
            d2 = d2.clamp(min=0)
            out = d2.sqrt() if sqrt_out else d2
        if zero_diagonal:
            out = out.masked_fill(eye, 0.0)
        return out if batched else out[0]
    if kind == 3:
        v = (dot.double() * scale + coef) ** degree
        if zero_diagonal:
            v = v.masked_fill(eye, 0.0)
        v = v.sum((1, 2)).reshape(b, 1)  # one "partial" per batch
        return v if batched else v[0]
    tiles = -(-m // _GEMM_TILE)
    pad = tiles * _GEMM_TILE - m
    if kind == 6:  # row partials [b, n, tiles_m] | column partials [b, tiles_n, m], flattened
        tn = -(-n // _GEMM_TILE)
        v = dot * scale
        rows = torch.nn.functional.pad(v, (0, pad), value=-3.0e38).reshape(b, n, tiles, _GEMM_TILE).amax(-1)
        cols = torch.nn.functional.pad(v, (0, 0, 0, tn * _GEMM_TILE - n), value=-3.0e38)
        cols = cols.reshape(b, tn, _GEMM_TILE, m).amax(2)
        return torch.cat([rows.reshape(-1), cols.reshape(-1)])
    if kind == 4:
        v = 1.0 - (dot * aux_x.reshape(b, n, 1).float() * aux_y.reshape(b, 1, m).float()).abs()
        v = torch.nn.functional.pad(v, (0, pad), value=3.0e38)
        v = v.reshape(b, n, tiles, _GEMM_TILE).amin(-1)
        return v if batched else v[0]
    v = torch.nn.functional.pad(dot * scale, (0, pad))
    v = v.reshape(b, n, tiles, _GEMM_TILE).sum(-1)
    return v if batched else v[0]


def mc_bootstrap_update(preds: Tensor, target: Tensor, weights: Tensor, ws: Tensor, flag: Tensor, num_classes: int,
                        ignore_index: Optional[int]) -> None:
    """Host contract of ``csrc/classification/bootstrap.hip``: weighted [B, 3C+1] stat workspace per bootstrap."""
    C = int(num_classes)
    t = target.reshape(-1).long()
    p = preds.reshape(t.numel(), C).argmax(1) if preds.is_floating_point() else preds.reshape(-1).long()
    keep = torch.ones_like(t, dtype=torch.bool) if ignore_index is None else t != ignore_index
    bad_t = keep & ((t < 0) | (t >= C))
    bad_p = keep & ~bad_t & ((p < 0) | (p >= C))
    if bool(bad_t.any()):
        flag.view(-1)[0] |= 1
    if bool(bad_p.any()):
        flag.view(-1)[0] |= 2
    keep = keep & ~bad_t & ~bad_p
    w = weights.long().t() * keep  # [B, n]
    B = w.shape[0]
    stride = 3 * C + 1
    flat = ws.view(-1)
    base = (torch.arange(B) * stride).unsqueeze(1)
    tt, pp = t.clamp(0, C - 1), p.clamp(0, C - 1)
    hit = (pp == tt).unsqueeze(0)
    flat.index_add_(0, (base + tt).reshape(-1), (w * hit).reshape(-1))
    flat.index_add_(0, (base + C + pp).reshape(-1), (w * ~hit).reshape(-1))
    flat.index_add_(0, (base + 2 * C + tt).reshape(-1), (w * ~hit).reshape(-1))


# ------------------------------------------------------------------------------------------------------ RLE masks
def rle_encode(masks):
    """Host contract of ``tm_amd::rle_encode``: per image ``[n, H, W, areas, offsets(n+1), change positions]``.
    Change positions are the column-major indices where a mask flips value (starting from background)."""
    packs = []
    for m in masks:
        n, h, w = m.shape
        cm = m.detach().cpu().ne(0).transpose(1, 2).reshape(n, h * w).to(torch.int8)
        prev = torch.cat([torch.zeros(n, 1, dtype=torch.int8), cm[:, :-1]], 1)
        mi, pos = torch.nonzero(cm != prev, as_tuple=True)
        counts = torch.bincount(mi, minlength=n)
        off = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(counts, 0)])
        head = torch.tensor([n, h, w], dtype=torch.long)
        packs.append(torch.cat([head, cm.sum(1, dtype=torch.long), off, pos]).to(torch.int32).to(m.device))
    return packs


def rle_iou(dbuf, ddesc, gbuf, gdesc, pd, pg, gcrowd):
    out = torch.empty(pd.numel(), dtype=torch.float64)
    db, gb, dd, gd = dbuf.cpu().tolist(), gbuf.cpu().tolist(), ddesc.cpu().tolist(), gdesc.cpu().tolist()
    crowd = gcrowd.cpu().tolist()

    def intervals(buf, row):
        s, k, hw = row[0], row[1], row[3] * row[4]
        pts = buf[s:s + k] + ([hw] if k % 2 else [])
        return list(zip(pts[0::2], pts[1::2]))

    for p, (d, g) in enumerate(zip(pd.cpu().tolist(), pg.cpu().tolist())):
        a, b = dd[d], gd[g]
        if a[3] != b[3] or a[4] != b[4]:
            out[p] = -1.0
            continue
        ia, ib = intervals(db, a), intervals(gb, b)
        i = j = inter = 0
        while i < len(ia) and j < len(ib):
            lo, hi = max(ia[i][0], ib[j][0]), min(ia[i][1], ib[j][1])
            inter += max(0, hi - lo)
            if ia[i][1] < ib[j][1]:
                i += 1
            else:
                j += 1
        union = a[2] if crowd[g] else a[2] + b[2] - inter
        out[p] = inter / union if inter else 0.0
    return out.to(pd.device)


def box_pairwise_ragged(a: Tensor, b: Tensor, a_off: Tensor, b_off: Tensor, o_off: Tensor, a_lab: Tensor, b_lab: Tensor,
                        op: int, threshold, invalid: float) -> Tensor:
    """Host twin of the ragged IoU-family kernel: image by image (CPU tensors)."""
    ao, bo = a_off.tolist(), b_off.tolist()
    parts = []
    for i in range(len(ao) - 1):
        mat = box_pairwise(a[ao[i]:ao[i + 1]], b[bo[i]:bo[i + 1]], op, False)
        if threshold is not None:
            mat = torch.where(mat < threshold, torch.full_like(mat, invalid), mat)
        if a_lab.numel() or b_lab.numel():
            same = a_lab[ao[i]:ao[i + 1]].unsqueeze(1) == b_lab[bo[i]:bo[i + 1]].unsqueeze(0)
            mat = torch.where(same, mat, torch.full_like(mat, invalid))
        parts.append(mat.reshape(-1))
    dt = a.dtype if a.is_floating_point() else torch.float32
    return torch.cat(parts) if parts else torch.zeros(0, dtype=dt)


def iou_class_reduce(vals: Tensor, o_off: Tensor, b_off: Tensor, gt_lab: Tensor, classes: Tensor, invalid: float):
    """Host twin of ``iou_class_reduce_kernel`` (vectorised over all images)."""
    K = classes.numel()
    sums = torch.zeros(K + 1, dtype=torch.float64)
    counts = torch.zeros(K + 1, dtype=torch.int64)
    sizes, m = o_off.diff(), b_off.diff()
    img = torch.repeat_interleave(torch.arange(sizes.numel()), sizes)
    valid = vals != invalid
    v = vals[valid].double()
    sums[K] = v.sum()
    counts[K] = int(valid.sum())
    if K:
        local = torch.arange(vals.numel()) - o_off[img]
        lab = gt_lab[b_off[img] + local % m[img].clamp(min=1)][valid]
        k = torch.searchsorted(classes, lab)
        sums[:K] = torch.zeros(K, dtype=torch.float64).index_add_(0, k, v)
        counts[:K] = torch.bincount(k, minlength=K)
    return sums, counts


_NARROW_WIRES = ((torch.uint8, 255), (torch.float16, 2048), (torch.int32, 2**31 - 1))


def narrow_encode(src: Tensor, code: int, world: int) -> Tensor:
    """Host twin of ``narrow_encode_kernel``: values in the wire dtype + [too big, negative] check slots."""
    dtype, wmax = _NARROW_WIRES[code]
    if src.dtype == torch.int32 and code == 2:
        raise RuntimeError("narrow_encode: an int32 source is not narrowed to int32")
    wire = torch.zeros(src.numel() + 2, dtype=dtype)
    flat = src.reshape(-1)
    if flat.numel():
        wire[:-2] = flat.to(dtype)
        wire[-2] = int(bool((flat > wmax // world).any()))
        wire[-1] = int(bool((flat < 0).any()))
    return wire


def narrow_decode(wire: Tensor, n: int, out_dtype: torch.dtype, word: Optional[Tensor], bit: int) -> Tensor:
    if word is not None and bool((wire[n:] != 0).any()):
        word.bitwise_or_(bit)
    return wire[:n].to(out_dtype)
