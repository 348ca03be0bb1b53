"""Incremental calibration bins (``classification/extras.py`` ``_BinnedCalibration``) on the GPU.

The cached bins must give the CPU list-state result after many updates, after ``forward()`` merges, resets,
state-dict loads and under a 2-rank sync (bins all-reduced instead of lists gathered)."""
import pytest
import torch

from torchmetrics_amd.classification import BinaryCalibrationError, MulticlassCalibrationError
from tests.helpers import assert_close, run_ddp

pytestmark = pytest.mark.gpu


def _batches(seed, n=6, m=4000, c=7):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(m, c, generator=g) * 2, torch.randint(0, c, (m,), generator=g)) for _ in range(n)]


@pytest.mark.parametrize("norm", ["l1", "max", "l2"])
@pytest.mark.parametrize("n_bins", [1, 15, 100])
def test_multiclass_cached_bins_match_cpu(norm, n_bins):
    gpu = MulticlassCalibrationError(7, n_bins=n_bins, norm=norm).cuda()
    cpu = MulticlassCalibrationError(7, n_bins=n_bins, norm=norm)
    for k, (p, t) in enumerate(_batches(n_bins)):
        gpu.update(p.cuda(), t.cuda())
        cpu.update(p, t)
        assert gpu.__dict__.get("_bin_cache") is not None
        if k % 2:  # compute every other step (the per-step-compute pattern), the cache keeps accumulating
            assert_close(gpu.compute().cpu(), cpu.compute(), atol=2e-6, rtol=1e-5)
    assert_close(gpu.compute().cpu(), cpu.compute(), atol=2e-6, rtol=1e-5)


@pytest.mark.parametrize("norm", ["l1", "max", "l2"])
def test_binary_cached_bins_match_cpu(norm):
    g = torch.Generator().manual_seed(3)
    gpu = BinaryCalibrationError(n_bins=10, norm=norm).cuda()
    cpu = BinaryCalibrationError(n_bins=10, norm=norm)
    for _ in range(5):
        p, t = torch.rand(3000, generator=g), torch.randint(0, 2, (3000,), generator=g)
        gpu.update(p.cuda(), t.cuda())
        cpu.update(p, t)
    assert_close(gpu.compute().cpu(), cpu.compute(), atol=2e-6, rtol=1e-5)


def test_cache_survives_forward_reset_and_state_loads():
    batches = _batches(11)
    gpu = MulticlassCalibrationError(7, n_bins=15).cuda()
    cpu = MulticlassCalibrationError(7, n_bins=15)
    for p, t in batches[:3]:
        assert_close(gpu(p.cuda(), t.cuda()).cpu(), cpu(p, t), atol=2e-6, rtol=1e-5)  # forward: batch value
    assert_close(gpu.compute().cpu(), cpu.compute(), atol=2e-6, rtol=1e-5)  # re-seeded from the merged lists
    gpu.update(*(x.cuda() for x in batches[3]))
    cpu.update(*batches[3])
    assert_close(gpu.compute().cpu(), cpu.compute(), atol=2e-6, rtol=1e-5)
    gpu.reset()
    cpu.reset()
    gpu.update(*(x.cuda() for x in batches[4]))
    cpu.update(*batches[4])
    assert_close(gpu.compute().cpu(), cpu.compute(), atol=2e-6, rtol=1e-5)
    # states written from outside: the element count no longer matches the cache -> re-bin from the lists
    gpu.confidences = [torch.rand(100, device="cuda")]
    gpu.accuracies = [torch.ones(100, device="cuda")]
    cpu.confidences = [gpu.confidences[0].cpu()]
    cpu.accuracies = [torch.ones(100)]
    gpu._computed = cpu._computed = None
    assert_close(gpu.compute().cpu(), cpu.compute(), atol=2e-6, rtol=1e-5)


def _ddp_body(rank, world):
    torch.cuda.set_device(0)
    batches = _batches(21, n=4)
    m = MulticlassCalibrationError(7, n_bins=15).cuda()
    for p, t in batches[rank::world]:
        m.update(p.cuda(), t.cuda())
    got = m.compute().cpu()
    assert len(m.confidences) in (1, 2)  # local lists untouched by the bins all-reduce
    ref = MulticlassCalibrationError(7, n_bins=15)
    for p, t in batches:
        ref.update(p, t)
    assert_close(got, ref.compute(), atol=2e-6, rtol=1e-5)


def test_cached_bins_two_ranks_one_device():
    run_ddp(_ddp_body)
