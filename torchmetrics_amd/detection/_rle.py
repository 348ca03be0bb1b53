"""Run-length encoded masks: packs, descriptors and the COCO ``segmentation`` formats.

A mask is held by its *change positions* -- the column-major (COCO order: ``x * H + y``) indices where the value flips,
starting from background -- i.e. COCO's RLE counts in cumulative form.  One image's masks are one int32 pack::

    [n, H, W, area_0 .. area_{n-1}, off_0 .. off_n, positions ...]

built on the device by ``ops.rle_encode`` (``csrc/detection/rle.hip``).  This replaces the reference's host
pycocotools round trip (``S/detection/mean_ap.py:825-829`` encode, ``:899-903`` areas, ``:1007-1038`` object gather):
packs are ordinary tensor list states, so the sync engine gathers them, and mask IoU is ``ops.rle_iou`` on the device.

The COCO string codec and the polygon rasteriser follow the public COCO mask API format (``rleToString`` /
``rleFrString`` / ``rleFrPoly`` semantics), so json files written here load in COCO tools and vice versa.
"""
import math
from typing import Any, Dict, List, Sequence, Tuple

import numpy as np
import torch
from torch import Tensor

from torchmetrics_amd import ops


def encode(masks: Sequence[Tensor]) -> List[Tensor]:
    """One pack per ``[n, H, W]`` mask tensor (bool / uint8 / any dtype: nonzero is foreground)."""
    return ops.rle_encode([m if m.dim() == 3 else m.reshape(0, 0, 0) for m in masks])


def descriptors(packs: Sequence[Tensor], counts: Sequence[int], device: torch.device) -> Tuple[Tensor, Tensor]:
    """Concatenate packs into one buffer and describe every mask (flat image order) by an int64 row
    ``[position start, change count, area, H, W]`` -- all gathers on the device, no host sync (the per-image mask
    counts ``counts`` are host metadata: the labels' lengths)."""
    if not packs:
        return torch.zeros(1, dtype=torch.int32, device=device), torch.zeros(0, 5, dtype=torch.long, device=device)
    buf = torch.cat([p.to(device=device, dtype=torch.int32).reshape(-1) for p in packs])
    sizes = [p.numel() for p in packs]
    bases_host = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    n_host = np.asarray(counts, dtype=np.int64)
    total = int(n_host.sum())
    if total == 0:
        return buf, torch.zeros(0, 5, dtype=torch.long, device=device)
    img = np.repeat(np.arange(len(packs)), n_host)
    local = np.arange(total) - np.repeat(np.cumsum(n_host) - n_host, n_host)
    meta = torch.from_numpy(np.stack([bases_host[img], n_host[img], local])).to(device)
    base, n, loc = meta[0], meta[1], meta[2]
    b = buf.long()
    area = b[base + 3 + loc]
    off = b[base + 3 + n + loc]
    k = b[base + 4 + n + loc] - off
    start = base + 4 + 2 * n + off
    return buf, torch.stack([start, k, area, b[base + 1], b[base + 2]], 1).contiguous()


def decode(pack: Tensor) -> Tensor:
    """``[n, H, W]`` bool masks of a pack (scatter the flips, cumulative parity)."""
    p = pack.long()
    n, h, w = (int(v) for v in p[:3].tolist())
    off = p[3 + n: 4 + 2 * n]
    pos = p[4 + 2 * n:]
    hw = h * w
    flips = torch.zeros(n, hw + 1, dtype=torch.int32, device=pack.device)
    if pos.numel():
        mask_of = torch.repeat_interleave(torch.arange(n, device=pack.device), off[1:] - off[:-1])
        flips.index_put_((mask_of, pos), torch.ones_like(pos, dtype=torch.int32), accumulate=True)
    cm = (torch.cumsum(flips[:, :hw], 1) % 2).bool()
    return cm.reshape(n, w, h).transpose(1, 2).contiguous()


# ----------------------------------------------------------------------------------------------- COCO formats
def positions_to_counts(pos: Sequence[int], hw: int) -> List[int]:
    """COCO counts (alternating background / foreground run lengths, background first) from change positions."""
    pts = [0, *pos, hw]
    return [b - a for a, b in zip(pts[:-1], pts[1:])]


def counts_to_positions(counts: Sequence[int]) -> List[int]:
    out, acc = [], 0
    for i, c in enumerate(counts):
        acc += int(c)
        if i < len(counts) - 1:
            out.append(acc)
    # zero-length runs produce repeated positions: a flip and its undo cancel
    dedup: List[int] = []
    for q in out:
        if dedup and dedup[-1] == q:
            dedup.pop()
        else:
            dedup.append(q)
    return dedup


def counts_to_string(counts: Sequence[int]) -> str:
    """COCO compressed counts: 5-bit groups with a continuation bit, offset by 48; from the fourth count on each value
    is stored as the difference to the count two places before."""
    chars = []
    for i, c in enumerate(counts):
        x = int(c) - (int(counts[i - 2]) if i > 2 else 0)
        more = True
        while more:
            ch = x & 0x1F
            x >>= 5
            more = (x != -1) if (ch & 0x10) else (x != 0)
            if more:
                ch |= 0x20
            chars.append(chr(ch + 48))
    return "".join(chars)


def string_to_counts(s: str) -> List[int]:
    counts: List[int] = []
    p = 0
    while p < len(s):
        x, k, more = 0, 0, True
        while more:
            c = ord(s[p]) - 48
            x |= (c & 0x1F) << (5 * k)
            more = bool(c & 0x20)
            p += 1
            k += 1
            if not more and (c & 0x10):
                x |= -1 << (5 * k)
        if len(counts) > 2:
            x += counts[-2]
        counts.append(x)
    return counts


def polygon_to_counts(xy: Sequence[float], h: int, w: int) -> List[int]:
    """Rasterise one polygon (``[x0, y0, x1, y1, ...]``) to COCO counts: the boundary is walked on a 5x upsampled grid,
    the points where it crosses a pixel-column centre become column-major toggles."""
    scale = 5.0
    k = len(xy) // 2
    x = [int(scale * xy[2 * j] + 0.5) for j in range(k)]
    y = [int(scale * xy[2 * j + 1] + 0.5) for j in range(k)]
    x.append(x[0])
    y.append(y[0])
    u: List[int] = []
    v: List[int] = []
    for j in range(k):
        xs, xe, ys, ye = x[j], x[j + 1], y[j], y[j + 1]
        dx, dy = abs(xe - xs), abs(ys - ye)
        flip = (dx >= dy and xs > xe) or (dx < dy and ys > ye)
        if flip:
            xs, xe, ys, ye = xe, xs, ye, ys
        if dx >= dy:
            s = (ye - ys) / dx if dx else 0.0
            for d in range(dx + 1):
                t = dx - d if flip else d
                u.append(t + xs)
                v.append(int(ys + s * t + 0.5))
        else:
            s = (xe - xs) / dy if dy else 0.0
            for d in range(dy + 1):
                t = dy - d if flip else d
                v.append(t + ys)
                u.append(int(xs + s * t + 0.5))
    pts = []
    for j in range(1, len(u)):
        if u[j] == u[j - 1]:
            continue
        xd = float(u[j] if u[j] < u[j - 1] else u[j] - 1)
        xd = (xd + 0.5) / scale - 0.5
        if math.floor(xd) != xd or xd < 0 or xd > w - 1:
            continue
        yd = float(v[j] if v[j] < v[j - 1] else v[j - 1])
        yd = (yd + 0.5) / scale - 0.5
        yd = min(max(yd, 0.0), float(h))
        pts.append(int(xd) * h + int(math.ceil(yd)))
    pts.append(h * w)
    pts.sort()
    a, prev = [], 0
    for t in pts:
        a.append(t - prev)
        prev = t
    b = [a[0]]
    j = 1
    while j < len(a):
        if a[j] > 0:
            b.append(a[j])
            j += 1
        else:
            j += 1
            if j < len(a):
                b[-1] += a[j]
                j += 1
    return b


def segmentation_to_mask(segm: Any, h: int, w: int) -> np.ndarray:
    """``[H, W]`` uint8 mask of a COCO ``segmentation`` entry: polygons (list of lists, united), uncompressed RLE
    (``counts`` list) or compressed RLE (``counts`` string)."""
    if isinstance(segm, list):
        out = np.zeros((h, w), dtype=np.uint8)
        for poly in segm:
            out |= _counts_to_mask(polygon_to_counts(poly, h, w), h, w)
        return out
    if isinstance(segm, dict):
        sh, sw = (int(v) for v in segm.get("size", (h, w)))
        counts = segm["counts"]
        if isinstance(counts, bytes):
            counts = counts.decode("ascii")
        if isinstance(counts, str):
            counts = string_to_counts(counts)
        return _counts_to_mask(counts, sh, sw)
    raise ValueError(f"Unsupported COCO segmentation entry of type {type(segm)}")


def _counts_to_mask(counts: Sequence[int], h: int, w: int) -> np.ndarray:
    flat = np.zeros(h * w, dtype=np.uint8)
    acc, val = 0, 0
    for c in counts:
        if val:
            flat[acc: acc + int(c)] = 1
        acc += int(c)
        val ^= 1
    return flat.reshape(w, h).T.copy()


def pack_to_coco(pack: Tensor) -> List[Dict[str, Any]]:
    """COCO compressed-RLE ``segmentation`` dicts (``{"size": [H, W], "counts": str}``) of every mask of a pack."""
    p = pack.cpu().long().tolist()
    n, h, w = p[0], p[1], p[2]
    off = p[3 + n: 4 + 2 * n]
    pos = p[4 + 2 * n:]
    return [{"size": [h, w], "counts": counts_to_string(positions_to_counts(pos[off[i]: off[i + 1]], h * w))}
            for i in range(n)]
