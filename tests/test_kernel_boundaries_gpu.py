"""Both sides of every kernel-applicability boundary on the GPU give the CPU result.

The fused reductions take the HIP kernel up to a size limit and ATen device ops beyond it (``ops.confmat_reducible``:
C <= 4096 for kappa / MCC / Jaccard, LDS-resident row / column sums; ``ops.regression_computable``: <= 2^20 outputs
for the regression compute kernel).  Each test runs the limit and limit + 1 on the device and compares with the CPU
path (an independent op chain) on identical states.
"""
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification.cohen_kappa import _cohen_kappa_reduce
from torchmetrics_amd.functional.classification.jaccard import _jaccard_index_reduce
from torchmetrics_amd.functional.classification.matthews_corrcoef import _matthews_corrcoef_reduce
from torchmetrics_amd.regression import MeanSquaredError, PearsonCorrCoef, R2Score
from tests.helpers import assert_close

pytestmark = pytest.mark.gpu


def _confmat(c, n=400_000, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, c, (n,), generator=g)
    p = torch.where(torch.rand(n, generator=g) < 0.6, t, torch.randint(0, c, (n,), generator=g))
    return torch.bincount(t * c + p, minlength=c * c).reshape(c, c)


@pytest.mark.parametrize("c", [4096, 4097])
def test_confmat_reductions_at_the_kernel_limit(c):
    cm = _confmat(c)
    assert ops.confmat_reducible(cm.cuda()) == (c <= 4096)
    for weights in (None, "linear", "quadratic"):
        assert_close(_cohen_kappa_reduce(cm.cuda(), weights).cpu(), _cohen_kappa_reduce(cm, weights), atol=1e-5,
                     rtol=1e-4)
    assert_close(_matthews_corrcoef_reduce(cm.cuda()).cpu(), _matthews_corrcoef_reduce(cm), atol=1e-5, rtol=1e-4)
    for average in ("macro", "micro", "weighted", "none"):
        got = _jaccard_index_reduce(cm.cuda(), average=average).cpu()
        assert_close(got, _jaccard_index_reduce(cm, average=average), atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("k", [1 << 20, (1 << 20) + 1])
@pytest.mark.parametrize("cls", [MeanSquaredError, R2Score, PearsonCorrCoef])
def test_regression_compute_at_the_kernel_limit(cls, k):
    g = torch.Generator().manual_seed(1)
    preds = torch.randn(6, k, generator=g)
    target = preds + 0.3 * torch.randn(6, k, generator=g)
    kw = {"num_outputs": k}
    if cls is R2Score:
        kw = {"num_outputs": k, "multioutput": "raw_values"}
    gpu, cpu = cls(**kw).cuda(), cls(**kw)
    gpu.update(preds.cuda(), target.cuda())
    cpu.update(preds, target)
    states = [getattr(gpu, s) for s in gpu._defaults if isinstance(getattr(gpu, s), torch.Tensor)
              and getattr(gpu, s).numel() == k]
    if states:
        assert ops.regression_computable(states, 6) == (k <= 1 << 20)
    assert_close(gpu.compute().cpu(), cpu.compute(), atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("k", [255, 256, 257, 1000, 4099])
def test_moments_update_kernel_switch(k):
    """Up to 256 outputs the grid-stride moments kernel, beyond it the column-parallel one (rows split in chunks)."""
    g = torch.Generator().manual_seed(k)
    preds = torch.randn(3000, k, generator=g)
    target = preds + 0.5 * torch.randn(3000, k, generator=g)
    for cls, kw in ((MeanSquaredError, {}), (PearsonCorrCoef, {}), (R2Score, {"multioutput": "raw_values"})):
        gpu, cpu = cls(num_outputs=k, **kw).cuda(), cls(num_outputs=k, **kw)
        for lo in range(0, 3000, 1000):
            gpu.update(preds[lo:lo + 1000].cuda(), target[lo:lo + 1000].cuda())
            cpu.update(preds[lo:lo + 1000], target[lo:lo + 1000])
        assert_close(gpu.compute().cpu(), cpu.compute(), atol=1e-5, rtol=1e-4)
