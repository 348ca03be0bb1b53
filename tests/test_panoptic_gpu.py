"""Panoptic quality segment tables on the device (``csrc/detection/panoptic.hip``) vs the sort path on the CPU."""
import pytest
import torch

from torchmetrics_amd.functional.detection import modified_panoptic_quality, panoptic_quality
from torchmetrics_amd.functional.detection import panoptic_qualities as PQ
from tests.helpers import assert_close

pytestmark = pytest.mark.gpu

THINGS, STUFFS = {0, 1, 3}, {6, 7}


def _blocky(g, b, h, w, n_seg, noise=0.0):
    """Blocky panoptic maps: categories from THINGS | STUFFS (+ unknown 9), instances per block."""
    cats = torch.tensor(sorted(THINGS | STUFFS) + [9])
    bh, bw = max(1, h // n_seg), max(1, w // n_seg)
    yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    block = (yy // bh) * (w // bw + 1) + (xx // bw)
    out = torch.zeros(b, h, w, 2, dtype=torch.long)
    for i in range(b):
        perm = torch.randint(0, len(cats), (int(block.max()) + 1,), generator=g)
        inst = torch.randint(0, 4, (int(block.max()) + 1,), generator=g)
        out[i, ..., 0] = cats[perm][block]
        out[i, ..., 1] = inst[block]
        if noise:
            flip = torch.rand(h, w, generator=g) < noise
            out[i, ..., 0] = torch.where(flip, cats[torch.randint(0, len(cats), (h, w), generator=g)], out[i, ..., 0])
    return out


@pytest.mark.parametrize(("b", "h", "w", "n_seg"), [(1, 16, 16, 2), (4, 64, 80, 6), (2, 128, 96, 12), (3, 200, 200, 40)])
@pytest.mark.parametrize("fn", [panoptic_quality, modified_panoptic_quality])
def test_device_tables_match_cpu(b, h, w, n_seg, fn):
    g = torch.Generator().manual_seed(b * h + n_seg)
    target = _blocky(g, b, h, w, n_seg)
    preds = torch.roll(_blocky(g, b, h, w, n_seg, noise=0.05), shifts=2, dims=2)
    got = fn(preds.cuda(), target.cuda(), THINGS, STUFFS, allow_unknown_preds_category=True).cpu()
    want = fn(preds, target, THINGS, STUFFS, allow_unknown_preds_category=True)
    assert_close(got, want, atol=1e-9, rtol=1e-7)


def test_table_overflow_falls_back_to_sort_path():
    g = torch.Generator().manual_seed(0)
    # ~2500 distinct instances in one image: more segments than a per-image table holds
    target = torch.zeros(1, 100, 100, 2, dtype=torch.long)
    target[..., 0] = 0
    target[..., 1] = torch.arange(10000).reshape(100, 100) // 4
    preds = target.clone()
    preds[..., 1] = torch.roll(preds[..., 1], 1, dims=2)
    codes = PQ._device_segment_tables  # the helper returns None on overflow
    cat_tab = torch.tensor(sorted(THINGS | STUFFS) + [10], device="cuda")
    assert codes(preds.reshape(1, -1, 2).cuda(), target.reshape(1, -1, 2).cuda(), cat_tab, 2501, 5,
                 1 * 6 * 2501) is None
    got = panoptic_quality(preds.cuda(), target.cuda(), THINGS, STUFFS).cpu()
    want = panoptic_quality(preds, target, THINGS, STUFFS)
    assert_close(got, want, atol=1e-9, rtol=1e-7)
