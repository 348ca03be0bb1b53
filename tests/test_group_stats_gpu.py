"""Group stat-score kernel (``csrc/classification/group_stats.hip``) vs a per-group PyTorch computation of the
reference's formulation (``F/classification/group_fairness.py``: sigmoid-or-not, threshold, ignore_index, tp/fp/tn/fn
per group), through BinaryGroupStatRates / BinaryFairness on the GPU."""
import pytest
import torch

import torchmetrics_amd as tm

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _per_group(preds, target, groups, num_groups, threshold, ignore_index):
    if preds.is_floating_point():
        if not ((preds >= 0) & (preds <= 1)).all():
            preds = preds.sigmoid()
        preds = (preds > threshold).long()
    out = torch.zeros(num_groups, 4, dtype=torch.long)
    for g in range(num_groups):
        m = groups == g
        if ignore_index is not None:
            m &= target != ignore_index
        p, t = preds[m], target[m]
        out[g] = torch.stack([((p == 1) & (t == 1)).sum(), ((p == 1) & (t != 1)).sum(),
                              ((p != 1) & (t == 0)).sum(), ((p != 1) & (t != 0)).sum()])
    return out


@pytest.mark.parametrize("n", [1, 1000, 300_001])
@pytest.mark.parametrize("num_groups", [2, 7, 1500])
@pytest.mark.parametrize("reading", ["probs", "logits", "labels", "bf16_logits"])
@pytest.mark.parametrize("ignore_index", [None, -1])
def test_group_stats_match_per_group_formula(n, num_groups, reading, ignore_index):
    g = torch.Generator().manual_seed(n + num_groups)
    target = torch.randint(0, 2, (n,), generator=g)
    groups = torch.randint(0, num_groups, (n,), generator=g)
    if reading == "probs":
        preds = torch.rand(n, generator=g)
    elif reading == "labels":
        preds = torch.randint(0, 2, (n,), generator=g)
    else:
        preds = torch.randn(n, generator=g) * 3
        if reading == "bf16_logits":
            preds = preds.to(torch.bfloat16)
    if ignore_index is not None:
        target[torch.rand(n, generator=g) < 0.1] = ignore_index
    if reading == "bf16_logits" and not ((preds >= 0) & (preds <= 1)).all():
        # the sigmoid is rounded to bf16 before the threshold, as ATen computes it in the scores' dtype
        exp = _per_group(preds.float().sigmoid().to(torch.bfloat16).float(), target, groups, num_groups, 0.5,
                         ignore_index)
    else:
        exp = _per_group(preds.float() if reading == "bf16_logits" else preds, target, groups, num_groups, 0.5,
                         ignore_index)
    m = tm.BinaryGroupStatRates(num_groups, ignore_index=ignore_index, validate_args=False).to(DEV)
    half = n // 2
    for sl in (slice(0, half), slice(half, n)):
        m.update(preds[sl].to(DEV), target[sl].to(DEV), groups[sl].to(DEV))
    got = torch.stack([m.tp, m.fp, m.tn, m.fn], 1).cpu()
    assert torch.equal(got, exp)


def test_fairness_module_matches_cpu():
    g = torch.Generator().manual_seed(0)
    preds, target, groups = torch.rand(5000, generator=g), torch.randint(0, 2, (5000,), generator=g), \
        torch.randint(0, 3, (5000,), generator=g)
    gpu = tm.BinaryFairness(3).to(DEV)
    cpu = tm.BinaryFairness(3)
    gpu.update(preds.to(DEV), target.to(DEV), groups.to(DEV))
    cpu.update(preds, target, groups)
    out_g, out_c = gpu.compute(), cpu.compute()
    assert out_g.keys() == out_c.keys()
    for k in out_c:
        torch.testing.assert_close(out_g[k].cpu(), out_c[k])
