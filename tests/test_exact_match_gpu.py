"""Exact-match kernel (``csrc/classification/exact_match.hip``) vs plain PyTorch formulas of the reference's
semantics (``F/classification/exact_match.py``): argmax / sigmoid-or-not / threshold / ignore_index / all-positions
vote, global and samplewise, module and functional."""
import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd.functional.classification import multiclass_exact_match, multilabel_exact_match

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_multiclass(preds, target, ignore_index, samplewise):
    if preds.ndim == target.ndim + 1:
        preds = preds.float().argmax(1)
    preds, target = preds.reshape(preds.shape[0], -1), target.reshape(target.shape[0], -1)
    if ignore_index is not None:
        preds = torch.where(target == ignore_index, torch.full_like(preds, ignore_index), preds)
    ok = ((preds == target).sum(1) == preds.shape[1]).float()
    return ok if samplewise else ok.mean()


def _ref_multilabel(preds, target, threshold, ignore_index, samplewise):
    if preds.is_floating_point():
        if not ((preds >= 0) & (preds <= 1)).all():
            preds = preds.sigmoid()
        preds = (preds > threshold).long()
    n, l = preds.shape[:2]
    preds, target = preds.reshape(n, l, -1), target.reshape(n, l, -1)
    if ignore_index is not None:
        # reference test baseline (T/classification/test_exact_match.py:160-167): only the target is masked
        target = target.masked_fill(target == ignore_index, -1)
    ok = ((preds == target).sum(1) == l).float()  # [N, P]
    return ok.mean(1) if samplewise else ok.mean()


@pytest.mark.parametrize("shape", [(4096, 10), (257, 1000), (300, 7, 33), (64, 5, 4, 9)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ignore_index", [None, -1])
@pytest.mark.parametrize("samplewise", [False, True])
def test_multiclass_scores(shape, dtype, ignore_index, samplewise):
    if samplewise and len(shape) == 2:
        pytest.skip("samplewise needs extra dims")
    g = torch.Generator().manual_seed(sum(shape))
    n, c = shape[:2]
    preds = torch.randn(*shape, generator=g).to(dtype)
    tshape = (n,) + tuple(shape[2:])
    target = preds.float().argmax(1)
    flip = torch.rand(tshape, generator=g) < (0.02 if len(shape) > 2 else 0.3)
    target = torch.where(flip, torch.randint(0, c, tshape, generator=g), target)
    if ignore_index is not None:
        target[torch.rand(tshape, generator=g) < 0.05] = ignore_index
    avg = "samplewise" if samplewise else "global"
    exp = _ref_multiclass(preds, target, ignore_index, samplewise)
    got_f = multiclass_exact_match(preds.to(DEV), target.to(DEV), c, avg, ignore_index)
    torch.testing.assert_close(got_f.cpu().float(), exp)
    m = tm.MulticlassExactMatch(c, multidim_average=avg, ignore_index=ignore_index).to(DEV)
    half = n // 2
    m.update(preds[:half].to(DEV), target[:half].to(DEV))
    m.update(preds[half:].to(DEV), target[half:].to(DEV))
    torch.testing.assert_close(m.compute().cpu().float(), exp)


@pytest.mark.parametrize("shape", [(1000, 3), (333, 4, 17)])
@pytest.mark.parametrize("samplewise", [False, True])
def test_multiclass_labels(shape, samplewise):
    if samplewise and len(shape) == 2:
        pytest.skip("samplewise needs extra dims")
    g = torch.Generator().manual_seed(1)
    target = torch.randint(0, 3, shape, generator=g)
    preds = torch.where(torch.rand(shape, generator=g) < 0.1, torch.randint(0, 3, shape, generator=g), target)
    avg = "samplewise" if samplewise else "global"
    exp = _ref_multiclass(preds, target, None, samplewise)
    m = tm.MulticlassExactMatch(3, multidim_average=avg).to(DEV)
    m.update(preds.to(DEV), target.to(DEV))
    torch.testing.assert_close(m.compute().cpu().float(), exp)


@pytest.mark.parametrize("shape", [(5000, 6), (400, 3, 50), (128, 16, 2, 3)])
@pytest.mark.parametrize("reading", ["probs", "logits", "labels"])
@pytest.mark.parametrize("ignore_index", [None, -1, 0])
@pytest.mark.parametrize("samplewise", [False, True])
def test_multilabel(shape, reading, ignore_index, samplewise):
    if samplewise and len(shape) == 2:
        pytest.skip("samplewise needs extra dims")
    g = torch.Generator().manual_seed(len(shape) * 7 + 3)
    target = torch.randint(0, 2, shape, generator=g)
    noisy = torch.where(torch.rand(shape, generator=g) < 0.01, 1 - target, target).float()
    if reading == "probs":
        preds = (noisy * 0.6 + 0.2 + 0.1 * torch.rand(shape, generator=g)).clamp(0, 1)
    elif reading == "logits":
        preds = (noisy * 2 - 1) * 3 + torch.randn(shape, generator=g)
    else:
        preds = noisy.long()
    if ignore_index == -1:
        target[torch.rand(shape, generator=g) < 0.05] = ignore_index
    avg = "samplewise" if samplewise else "global"
    exp = _ref_multilabel(preds, target, 0.5, ignore_index, samplewise)
    got = multilabel_exact_match(preds.to(DEV), target.to(DEV), shape[1], 0.5, avg, ignore_index)
    torch.testing.assert_close(got.cpu().float(), exp)
    m = tm.MultilabelExactMatch(shape[1], multidim_average=avg, ignore_index=ignore_index).to(DEV)
    for k in range(3):  # several updates: the prob-or-logit decision is per batch
        m.update(preds.to(DEV), target.to(DEV))
    torch.testing.assert_close(m.compute().cpu().float(), exp.repeat(3) if samplewise else exp)


def test_module_matches_cpu_module():
    g = torch.Generator().manual_seed(5)
    preds = torch.randn(777, 9, 5, generator=g)
    target = torch.randint(0, 9, (777, 5), generator=g)
    gpu = tm.MulticlassExactMatch(9).to(DEV)
    cpu = tm.MulticlassExactMatch(9)
    for sl in (slice(0, 300), slice(300, 777)):
        gpu.update(preds[sl].to(DEV), target[sl].to(DEV))
        cpu.update(preds[sl], target[sl])
    assert torch.equal(gpu.correct.cpu(), cpu.correct.reshape(gpu.correct.shape))
    assert torch.equal(gpu.total.cpu(), cpu.total.reshape(gpu.total.shape))
