"""Multilabel ranking kernel (``csrc/classification/ranking.hip``) vs scikit-learn and the CPU path."""
import numpy as np
import pytest
import torch
from sklearn.metrics import coverage_error, label_ranking_average_precision_score, label_ranking_loss

from torchmetrics_amd.classification import (
    MultilabelCoverageError,
    MultilabelRankingAveragePrecision,
    MultilabelRankingLoss,
)
from torchmetrics_amd.functional.classification import (
    multilabel_coverage_error,
    multilabel_ranking_average_precision,
    multilabel_ranking_loss,
)
from tests.helpers import assert_close

pytestmark = pytest.mark.gpu

SK = {multilabel_coverage_error: coverage_error,
      multilabel_ranking_average_precision: label_ranking_average_precision_score,
      multilabel_ranking_loss: label_ranking_loss}


@pytest.mark.parametrize("fn", list(SK), ids=lambda f: f.__name__)
@pytest.mark.parametrize(("n", "labels"), [(1, 2), (37, 5), (500, 64), (200, 300), (16, 2048)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_ranking_kernel_vs_sklearn(fn, n, labels, dtype):
    g = torch.Generator().manual_seed(n * labels)
    preds = torch.rand(n, labels, generator=g, dtype=torch.float64).to(dtype)
    target = torch.randint(0, 2, (n, labels), generator=g)
    if n > 2:
        target[0] = 0  # degenerate rows: no relevant / all relevant labels
        target[1] = 1
    got = fn(preds.cuda(), target.cuda(), num_labels=labels).cpu()
    want = SK[fn](target.numpy(), preds.double().numpy())
    assert_close(got, torch.tensor(want, dtype=torch.float32), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("fn", [multilabel_coverage_error, multilabel_ranking_average_precision],
                         ids=lambda f: f.__name__)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_ranking_kernel_ties_and_low_precision_match_cpu(fn, dtype):
    g = torch.Generator().manual_seed(5)
    preds = (torch.randint(0, 6, (300, 17), generator=g).float() / 5).to(dtype)  # many ties
    target = torch.randint(0, 2, (300, 17), generator=g)
    assert_close(fn(preds.cuda(), target.cuda(), num_labels=17).cpu(), fn(preds, target, num_labels=17),
                 atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("cls", [MultilabelCoverageError, MultilabelRankingAveragePrecision, MultilabelRankingLoss])
def test_ranking_modules_ignore_index_match_cpu(cls):
    g = torch.Generator().manual_seed(9)
    gpu, cpu = cls(num_labels=12, ignore_index=-1).cuda(), cls(num_labels=12, ignore_index=-1)
    for _ in range(3):
        preds = torch.randn(64, 12, generator=g)  # logits: sigmoid applied by the format step
        target = torch.randint(-1, 2, (64, 12), generator=g)
        gpu.update(preds.cuda(), target.cuda())
        cpu.update(preds, target)
    assert_close(gpu.compute().cpu(), cpu.compute(), atol=1e-5, rtol=1e-5)
