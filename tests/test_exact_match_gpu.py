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


@pytest.fixture
def no_torch_body(monkeypatch):
    """Every ROCm input below must be served by exact_match.hip: the torch update bodies raise if reached."""
    import torchmetrics_amd.classification.extras as ex
    import torchmetrics_amd.functional.classification.exact_match as fx

    def boom(*a, **k):
        raise AssertionError("ATen exact-match body reached on ROCm inputs")

    for mod in (ex, fx):
        for name in ("_multiclass_exact_match_update", "_multilabel_exact_match_update"):
            if hasattr(mod, name):
                monkeypatch.setattr(mod, name, boom)


@pytest.mark.parametrize("shape", [(1000, 3), (333, 4, 17)])
@pytest.mark.parametrize("samplewise", [False, True])
@pytest.mark.parametrize("ignore_index", [None, -1, 1])
@pytest.mark.parametrize("pdtype", [torch.int64, torch.int32, torch.float32, torch.bfloat16])
def test_multiclass_labels(shape, samplewise, ignore_index, pdtype, no_torch_body):
    if samplewise and len(shape) == 2:
        pytest.skip("samplewise needs extra dims")
    g = torch.Generator().manual_seed(1)
    target = torch.randint(0, 3, shape, generator=g)
    preds = torch.where(torch.rand(shape, generator=g) < 0.1, torch.randint(0, 3, shape, generator=g), target)
    if ignore_index == -1:
        target[torch.rand(shape, generator=g) < 0.05] = ignore_index
    preds = preds.to(pdtype)
    if pdtype.is_floating_point:  # float labels (validate_args=False): non-integral values never match
        preds = torch.where(torch.rand(shape, generator=g) < 0.02, preds + 0.5, preds)
    avg = "samplewise" if samplewise else "global"
    exp = _ref_multiclass(preds, target, ignore_index, samplewise)
    m = tm.MulticlassExactMatch(3, multidim_average=avg, ignore_index=ignore_index,
                                validate_args=not pdtype.is_floating_point).to(DEV)
    m.update(preds.to(DEV), target.to(DEV))
    torch.testing.assert_close(m.compute().cpu().float(), exp)
    got_f = multiclass_exact_match(preds.to(DEV), target.to(DEV), 3, avg, ignore_index, validate_args=False)
    torch.testing.assert_close(got_f.cpu().float(), exp)


def test_degenerate_shapes_closed_form(no_torch_body):
    """Empty batches and zero-size position dims give the reference's torch results (worked out by hand from
    ``F/classification/exact_match.py``: a vote over zero positions is vacuously correct)."""
    L = torch.long
    cases = [  # (preds, target, multilabel, avg, expected sum of correct, expected total)
        (torch.randn(0, 5), torch.zeros(0, dtype=L), False, "global", 0, 0),
        (torch.randn(4, 5, 0), torch.zeros(4, 0, dtype=L), False, "global", 4, 4),
        (torch.randn(4, 5, 0), torch.zeros(4, 0, dtype=L), False, "samplewise", 4, 1),
        (torch.zeros(4, 0, dtype=L), torch.zeros(4, 0, dtype=L), False, "global", 4, 4),
        (torch.rand(0, 3), torch.zeros(0, 3, dtype=L), True, "global", 0, 0),
        (torch.rand(4, 3, 0), torch.zeros(4, 3, 0, dtype=L), True, "global", 0, 0),
        (torch.rand(4, 3, 0), torch.zeros(4, 3, 0, dtype=L), True, "samplewise", 0, 0),
    ]
    for preds, target, ml, avg, exp_c, exp_t in cases:
        cls = tm.MultilabelExactMatch if ml else tm.MulticlassExactMatch
        m = cls(3 if ml else 5, multidim_average=avg, validate_args=False).to(DEV)
        m.update(preds.to(DEV), target.to(DEV))
        correct = torch.cat(m.correct) if isinstance(m.correct, list) else m.correct
        assert int(correct.sum()) == exp_c and int(m.total.sum()) == exp_t, (preds.shape, ml, avg)


@pytest.mark.parametrize("samplewise", [False, True])
def test_float_target_compared_exactly(samplewise):
    """A floating target is compared as-is: target 1.5 matches preds 1.5 and nothing else, as the
    reference's ``preds == target`` does -- the labels kernel would truncate it, so those batches take the torch
    body."""
    target = torch.tensor([[1.5, 2.0], [0.0, 1.0], [1.5, 1.5], [2.0, 0.5]])
    preds = torch.tensor([[1.5, 2.0], [0.0, 1.0], [1.0, 1.5], [2.0, 0.0]])
    avg = "samplewise" if samplewise else "global"
    exp = _ref_multiclass(preds, target, None, samplewise)
    assert float(exp.sum()) == 2.0 if samplewise else float(exp) == 0.5
    got = multiclass_exact_match(preds.to(DEV), target.to(DEV), 3, avg, validate_args=False)
    torch.testing.assert_close(got.cpu().float(), exp)
    m = tm.MulticlassExactMatch(3, multidim_average=avg, validate_args=False).to(DEV)
    m.update(preds.to(DEV), target.to(DEV))
    torch.testing.assert_close(m.compute().cpu().float(), exp)
