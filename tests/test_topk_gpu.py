"""Top-k class labels (``csrc/classification/topk.hip``) against a stable fp32 sort, and top_k > 1 stat scores on the
GPU against the CPU path.

The kernel's order is (score descending, NaN highest, ties to the smaller column) -- exactly a stable descending
``torch.sort`` of the fp32 scores, so the comparison is exact, ties (bf16 / f16 / integer-valued scores) included.
"""
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.classification import MulticlassAccuracy, MulticlassF1Score, MulticlassStatScores
from tests.helpers import assert_close

pytestmark = pytest.mark.gpu


def _reference(x, k):
    return torch.sort(x.float(), dim=1, descending=True, stable=True).indices[:, :k].int()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize(("n", "c", "k"), [(1, 2, 2), (7, 5, 5), (1000, 10, 3), (513, 64, 16), (300, 65, 7),
                                           (64, 1000, 5), (9, 50_000, 16), (4099, 100, 2)])
def test_topk_labels_matches_stable_sort(dtype, n, c, k):
    g = torch.Generator().manual_seed(n * 31 + c + k)
    x = torch.randn(n, c, generator=g).to(dtype)
    got = ops.topk_labels(x.cuda(), k)
    assert got is not None and got.dtype == torch.int32 and got.shape == (n, k)
    assert torch.equal(got.cpu(), _reference(x, k))


def test_topk_labels_ties_and_nan():
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 4, (2000, 300), generator=g).float()  # heavy ties
    x[::7, 13] = float("nan")
    x[::11, 200] = float("nan")
    x[::13] = float("-inf")
    for k in (1, 4, 16):
        assert torch.equal(ops.topk_labels(x.cuda(), k).cpu(), _reference(x, k))


def test_topk_labels_not_applicable():
    x = torch.randn(4, 20)
    assert ops.topk_labels(x, 2) is None  # CPU
    assert ops.topk_labels(x.cuda(), 17) is None  # k > 16
    assert ops.topk_labels(x.double().cuda(), 2) is None
    assert ops.topk_labels(x.cuda(), 0) is None


@pytest.mark.parametrize("top_k", [2, 5])
@pytest.mark.parametrize("average", ["micro", "macro", "weighted", "none"])
def test_top_k_stat_scores_gpu_vs_cpu(top_k, average):
    g = torch.Generator().manual_seed(top_k)
    preds = torch.randn(5000, 37, generator=g).softmax(1)
    target = torch.randint(0, 37, (5000,), generator=g)
    for cls in (MulticlassAccuracy, MulticlassF1Score):
        gpu = cls(num_classes=37, top_k=top_k, average=average).cuda()
        cpu = cls(num_classes=37, top_k=top_k, average=average)
        for lo in range(0, 5000, 1250):
            gpu.update(preds[lo:lo + 1250].cuda(), target[lo:lo + 1250].cuda())
            cpu.update(preds[lo:lo + 1250], target[lo:lo + 1250])
        assert_close(gpu.compute().cpu(), cpu.compute(), atol=1e-6, rtol=1e-5)
    gpu = MulticlassStatScores(num_classes=37, top_k=top_k, average=None, ignore_index=3).cuda()
    cpu = MulticlassStatScores(num_classes=37, top_k=top_k, average=None, ignore_index=3)
    gpu.update(preds.cuda(), target.cuda())  # fp32: no score ties, so the CPU topk's tie order never matters
    cpu.update(preds, target)
    assert torch.equal(gpu.compute().cpu(), cpu.compute())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize(("n", "c", "k"), [(3000, 1000, 5), (777, 37, 3), (64, 20_000, 16), (50, 12, 12)])
def test_fused_topk_stats_match_label_path(dtype, n, c, k):
    """The fused kernel's workspace equals topk labels (the kernel's own order) + the mc_update label histogram."""
    g = torch.Generator().manual_seed(c + k)
    x = torch.randn(n, c, generator=g).to(dtype).cuda()
    t = torch.randint(0, c, (n,), generator=g).cuda()
    t[::9] = 1  # some ignored rows
    for samplewise in (False, True):
        size = (n if samplewise else 1) * (3 * c + 1)
        ws_fused = torch.zeros(size, dtype=torch.int64, device="cuda")
        ws_label = torch.zeros_like(ws_fused)
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        assert ops.mc_topk_update(x, t, ws_fused, flag, k, 1, samplewise)
        ops.mc_update(ops.topk_labels(x, k), t, ws_label, flag, c, 1, ops.MC_STATS, samplewise)
        assert torch.equal(ws_fused.cpu(), ws_label.cpu())
        assert int(flag.item()) == 0


def test_fused_topk_stats_flags_bad_target():
    x = torch.randn(100, 10, device="cuda")
    t = torch.randint(0, 10, (100,), device="cuda")
    t[17] = 10
    ws = torch.zeros(31, dtype=torch.int64, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert ops.mc_topk_update(x, t, ws, flag, 3, None, False)
    assert int(flag.item()) != 0
    assert int(ws[:10].sum() + ws[20:30].sum()) == 99  # rows counted = tp + fn (the last slot is unused)
