"""Distributed sync across every domain (reference model: ``run_ddp`` cases in ``T/unittests/**``).

Each case is run on a 2-rank gloo pool: rank r updates its metric with batches r, r+2, ...; the synced ``compute()``
must equal a single-process metric fed all batches.  This exercises every state kind the engine moves: sum/mean/
max/min tensors (all_reduce), ``cat`` lists of uneven length (one header + one payload all_gather), ``None`` lists
(element interleave), custom merges (Pearson), and python-object / string-derived states (text metrics keep tensors).
The single-process values are themselves pinned by the oracle / golden tests of each domain.
"""
import pytest
import torch

import torchmetrics_amd as tm
import torchmetrics_amd.audio
import torchmetrics_amd.clustering
import torchmetrics_amd.image
import torchmetrics_amd.text
import torchmetrics_amd.wrappers
from tests.helpers import assert_close, run_ddp

N_BATCH = 4


class _TinyFeatures(torch.nn.Module):
    """Stand-in feature extractor (FID / KID / IS accept any Module): per-channel mean and max -> 6 features."""

    def forward(self, x):
        x = x.float() / 32.0  # moderate logits: IS's softmax must not underflow to exact zeros
        return torch.cat([x.mean(dim=(2, 3)), x.amax(dim=(2, 3))], dim=1)


def _feat_batch(i):
    return torch.randint(0, 255, (8, 3, 6, 6), dtype=torch.uint8, generator=torch.Generator().manual_seed(i)), i % 2 == 0


def _images(seed, n=3, c=3, h=24, w=24):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(n, c, h, w, generator=g), torch.rand(n, c, h, w, generator=g)


def _signals(seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(3, 2, 800, generator=g)
    return 0.7 * t + 0.3 * torch.randn(3, 2, 800, generator=g), t


def _labels(seed, n=30, k=4):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, k, (n,), generator=g), torch.randint(0, k, (n,), generator=g)


_SENTENCES = [
    ("the cat sat on the mat", "a cat sat on the mat"),
    ("there is a dog in the house", "the dog is in the house"),
    ("hello world", "hello there world"),
    ("metrics on many gpus", "metrics on many devices"),
    ("one two three four", "one two four"),
    ("the quick brown fox", "the fast brown fox jumps"),
    ("a b c d e", "a b c d e"),
    ("sync the states", "synchronise all states"),
]


def _text(i):
    p = [_SENTENCES[(2 * i) % 8][0], _SENTENCES[(2 * i + 1) % 8][0]]
    t = [_SENTENCES[(2 * i) % 8][1], _SENTENCES[(2 * i + 1) % 8][1]]
    return p, t


# name -> (metric factory, batch(i) -> update args, compare tolerance[, single-process factory])
CASES = {
    # image
    "ssim": (lambda: tm.image.StructuralSimilarityIndexMeasure(data_range=1.0), _images, 1e-5),
    "psnr": (lambda: tm.image.PeakSignalNoiseRatio(data_range=1.0), _images, 1e-4),
    "uqi": (lambda: tm.image.UniversalImageQualityIndex(), _images, 1e-5),
    "tv": (lambda: tm.image.TotalVariation(), lambda i: (_images(i)[0],), 1e-3),
    "fid_features": (lambda: tm.image.FrechetInceptionDistance(feature=_TinyFeatures()), _feat_batch, 1e-3),
    "kid_features": (lambda: tm.image.KernelInceptionDistance(feature=_TinyFeatures(), subsets=3, subset_size=4),
                     _feat_batch, None),
    "inception_score": (lambda: tm.image.InceptionScore(feature=_TinyFeatures(), splits=2),
                        lambda i: (_feat_batch(i)[0],), None),
    # text
    "wer": (lambda: tm.text.WordErrorRate(), _text, 1e-6),
    "cer": (lambda: tm.text.CharErrorRate(), _text, 1e-6),
    "mer": (lambda: tm.text.MatchErrorRate(), _text, 1e-6),
    "bleu": (lambda: tm.text.BLEUScore(), lambda i: (_text(i)[0], [[r] for r in _text(i)[1]]), 1e-6),
    "sacrebleu": (lambda: tm.text.SacreBLEUScore(), lambda i: (_text(i)[0], [[r] for r in _text(i)[1]]), 1e-6),
    "chrf": (lambda: tm.text.CHRFScore(), lambda i: (_text(i)[0], [[r] for r in _text(i)[1]]), 1e-6),
    "ter": (lambda: tm.text.TranslationEditRate(), lambda i: (_text(i)[0], [[r] for r in _text(i)[1]]), 1e-6),
    "eed": (lambda: tm.text.ExtendedEditDistance(), _text, 1e-6),
    "rouge": (lambda: tm.text.ROUGEScore(), _text, 1e-6),
    "edit": (lambda: tm.text.EditDistance(), _text, 1e-6),
    "wil": (lambda: tm.text.WordInfoLost(), _text, 1e-6),
    "wip": (lambda: tm.text.WordInfoPreserved(), _text, 1e-6),
    "perplexity": (lambda: tm.text.Perplexity(ignore_index=0),
                   lambda i: (torch.randn(2, 7, 11, generator=torch.Generator().manual_seed(i)),
                              torch.randint(0, 11, (2, 7), generator=torch.Generator().manual_seed(i + 50))), 1e-5),
    "squad": (lambda: tm.text.SQuAD(),
              lambda i: ([{"prediction_text": _SENTENCES[i][0], "id": str(i)}],
                         [{"answers": {"answer_start": [0], "text": [_SENTENCES[i][1]]}, "id": str(i)}]), 1e-5),
    # regression states with custom merges (Pearson's moment merge) and cat lists (Spearman / Kendall)
    "pearson": (lambda: tm.PearsonCorrCoef(), lambda i: tuple(_signals(i)[k][0, 0, :50] for k in (0, 1)), 1e-5),
    "spearman": (lambda: tm.SpearmanCorrCoef(), lambda i: tuple(_signals(i)[k][0, 0, :50] for k in (0, 1)), 1e-5),
    "kendall": (lambda: tm.KendallRankCorrCoef(), lambda i: tuple(_signals(i)[k][0, 0, :50] for k in (0, 1)), 1e-5),
    "r2": (lambda: tm.R2Score(), lambda i: tuple(_signals(i)[k][0, 0, :50] for k in (0, 1)), 1e-5),
    # audio
    "snr": (lambda: tm.audio.SignalNoiseRatio(), _signals, 1e-4),
    "si_sdr": (lambda: tm.audio.ScaleInvariantSignalDistortionRatio(), _signals, 1e-4),
    "sa_sdr": (lambda: tm.audio.SourceAggregatedSignalDistortionRatio(), _signals, 1e-4),
    "pit": (lambda: tm.audio.PermutationInvariantTraining(tm.functional.audio.scale_invariant_signal_noise_ratio),
            _signals, 1e-4),
    # clustering (cat list states)
    "mutual_info": (lambda: tm.clustering.MutualInfoScore(), _labels, 1e-5),
    "adjusted_rand": (lambda: tm.clustering.AdjustedRandScore(), _labels, 1e-5),
    "fowlkes_mallows": (lambda: tm.clustering.FowlkesMallowsIndex(), _labels, 1e-5),
    # nominal (confmat sum states)
    "cramers_v": (lambda: tm.nominal.CramersV(num_classes=4), _labels, 1e-5),
    "theils_u": (lambda: tm.nominal.TheilsU(num_classes=4), _labels, 1e-5),
    "tschuprows_t": (lambda: tm.nominal.TschuprowsT(num_classes=4), _labels, 1e-5),
    # aggregation
    "mean": (lambda: tm.MeanMetric(), lambda i: (torch.arange(5.0) * (i + 1),), 1e-6),
    "sum": (lambda: tm.SumMetric(), lambda i: (torch.arange(5.0) * (i + 1),), 1e-6),
    "max": (lambda: tm.MaxMetric(), lambda i: (torch.arange(5.0) * (i + 1),), 1e-6),
    "min": (lambda: tm.MinMetric(), lambda i: (torch.arange(5.0) - i,), 1e-6),
    "cat": (lambda: tm.CatMetric(), lambda i: (torch.arange(i + 1.0),), "sorted"),
    # wrappers
    "minmax": (lambda: tm.MinMaxMetric(tm.MeanSquaredError()),
               lambda i: (torch.randn(6, generator=torch.Generator().manual_seed(i)), torch.zeros(6)), 1e-5),
    "multioutput": (lambda: tm.MultioutputWrapper(tm.MeanSquaredError(), num_outputs=2),
                    lambda i: (torch.randn(5, 2, generator=torch.Generator().manual_seed(i)), torch.zeros(5, 2)), 1e-5),
    # each rank's window holds both of its batches -> the synced window is every batch (a plain SumMetric)
    "running": (lambda: tm.wrappers.Running(tm.SumMetric(), window=2), lambda i: (torch.arange(5.0) * (i + 1),), 1e-6,
                tm.SumMetric),
    "multitask": (lambda: tm.MultitaskWrapper({"cls": tm.MulticlassAccuracy(num_classes=4), "reg": tm.MeanSquaredError()}),
                  lambda i: ({"cls": _labels(i)[0], "reg": _signals(i)[0][0, 0, :20]},
                             {"cls": _labels(i)[1], "reg": _signals(i)[1][0, 0, :20]}), 1e-5),
    "classwise": (lambda: tm.ClasswiseWrapper(tm.MulticlassAccuracy(num_classes=3, average=None)),
                  lambda i: _labels(i, 20, 3), 1e-6),
}


def _flatten(x):
    if isinstance(x, dict):
        return {k: _flatten(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_flatten(v) for v in x]
    return x


def _body(rank, world, name):
    factory, batch, tol = CASES[name][:3]
    single_factory = CASES[name][3] if len(CASES[name]) > 3 else factory
    torch.manual_seed(0)
    metric = factory()
    for i in range(rank, N_BATCH, world):
        metric.update(*batch(i))
    torch.manual_seed(123)
    got = metric.compute()
    single = single_factory()
    single.__dict__["_to_sync"] = False  # the reference value: one process, every batch
    for m in single.modules():
        if hasattr(m, "_to_sync"):
            m._to_sync = False
    for i in range(N_BATCH):
        single.update(*batch(i))
    torch.manual_seed(123)
    expect = single.compute()
    if tol == "sorted":
        assert_close(torch.sort(got.flatten()).values, torch.sort(expect.flatten()).values)
    elif tol is None:  # random subsets (KID): compare shapes and finiteness, the values are subset-dependent
        assert all(torch.isfinite(torch.as_tensor(v)).all() for v in got)
    else:
        assert_close(_flatten(got), _flatten(expect), atol=tol, rtol=tol)


@pytest.mark.parametrize("name", sorted(CASES))
def test_ddp_domain(name):
    run_ddp(_body, name)
