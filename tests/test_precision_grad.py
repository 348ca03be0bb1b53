"""Differentiability and reduced-precision support across domains.

Reference model: ``run_differentiability_test`` and ``run_precision_test_cpu/gpu`` in
``T/unittests/helpers/testers.py:476-578``: a metric's output requires grad exactly when the class declares
``is_differentiable``, differentiable functionals pass ``torch.autograd.gradcheck`` in fp64, and metrics accept
half / bfloat16 inputs (the output is a finite tensor).  Here the same checks run for one representative per family;
the GPU variants feed fp16 / bf16 CUDA inputs through the HIP kernels (which read 16-bit inputs natively).
"""
from functools import partial

import pytest
import torch

import torchmetrics_amd as tm
import torchmetrics_amd.audio
import torchmetrics_amd.functional as F
import torchmetrics_amd.image
import torchmetrics_amd.text  # noqa: F401

_g = torch.Generator().manual_seed(7)


def _t(*shape):
    return torch.rand(*shape, generator=_g)


def _n(*shape):
    return torch.randn(*shape, generator=_g)


def _i(hi, *shape):
    return torch.randint(0, hi, shape, generator=_g)


# name -> (module factory, functional or None, preds, target, half-ok on CPU)
CASES = {
    # regression
    "mse": (tm.MeanSquaredError, F.mean_squared_error, _n(12), _n(12)),
    "mae": (tm.MeanAbsoluteError, F.mean_absolute_error, _n(12), _n(12)),
    "msle": (tm.MeanSquaredLogError, F.mean_squared_log_error, _t(12), _t(12)),
    "mape": (tm.MeanAbsolutePercentageError, F.mean_absolute_percentage_error, _n(12), _n(12) + 3),
    "smape": (tm.SymmetricMeanAbsolutePercentageError, F.symmetric_mean_absolute_percentage_error, _n(12), _n(12)),
    "wmape": (tm.WeightedMeanAbsolutePercentageError, F.weighted_mean_absolute_percentage_error, _n(12), _n(12)),
    "r2": (tm.R2Score, F.r2_score, _n(12), _n(12)),
    "explained_variance": (tm.ExplainedVariance, F.explained_variance, _n(12), _n(12)),
    "pearson": (tm.PearsonCorrCoef, F.pearson_corrcoef, _n(12), _n(12)),
    "concordance": (tm.ConcordanceCorrCoef, F.concordance_corrcoef, _n(12), _n(12)),
    "spearman": (tm.SpearmanCorrCoef, F.spearman_corrcoef, _n(12), _n(12)),
    "kendall": (tm.KendallRankCorrCoef, F.kendall_rank_corrcoef, _n(12), _n(12)),
    "cosine": (tm.CosineSimilarity, F.cosine_similarity, _n(4, 6), _n(4, 6)),
    "log_cosh": (tm.LogCoshError, F.log_cosh_error, _n(12), _n(12)),
    "tweedie": (partial(tm.TweedieDevianceScore, power=1.5), partial(F.tweedie_deviance_score, power=1.5),
                _t(12) + 0.1, _t(12) + 0.1),
    "kl": (tm.KLDivergence, F.kl_divergence, torch.softmax(_n(4, 5), 1), torch.softmax(_n(4, 5), 1)),
    "minkowski": (partial(tm.MinkowskiDistance, p=3), partial(F.minkowski_distance, p=3), _n(12), _n(12)),
    "rse": (tm.RelativeSquaredError, F.relative_squared_error, _n(12), _n(12)),
    # classification (not differentiable: outputs never require grad)
    "binary_acc": (partial(tm.classification.BinaryAccuracy), F.classification.binary_accuracy, _t(20), _i(2, 20)),
    "mc_f1": (partial(tm.classification.MulticlassF1Score, num_classes=4),
              partial(F.classification.multiclass_f1_score, num_classes=4), _t(20, 4), _i(4, 20)),
    "ml_prec": (partial(tm.classification.MultilabelPrecision, num_labels=3),
                partial(F.classification.multilabel_precision, num_labels=3), _t(20, 3), _i(2, 20, 3)),
    "binary_auroc": (tm.classification.BinaryAUROC, F.classification.binary_auroc, _t(20), _i(2, 20)),
    "mc_ap": (partial(tm.classification.MulticlassAveragePrecision, num_classes=4),
              partial(F.classification.multiclass_average_precision, num_classes=4),
              torch.softmax(_n(20, 4), 1), _i(4, 20)),
    "mc_confmat": (partial(tm.classification.MulticlassConfusionMatrix, num_classes=4),
                   partial(F.classification.multiclass_confusion_matrix, num_classes=4), _t(20, 4), _i(4, 20)),
    "binary_calibration": (tm.classification.BinaryCalibrationError, F.classification.binary_calibration_error,
                           _t(20), _i(2, 20)),
    "mc_hinge": (partial(tm.classification.MulticlassHingeLoss, num_classes=4),
                 partial(F.classification.multiclass_hinge_loss, num_classes=4), _n(20, 4), _i(4, 20)),
    "mcc": (partial(tm.classification.MulticlassMatthewsCorrCoef, num_classes=4),
            partial(F.classification.multiclass_matthews_corrcoef, num_classes=4), _t(20, 4), _i(4, 20)),
    # audio
    "snr": (tm.audio.SignalNoiseRatio, F.audio.signal_noise_ratio, _n(2, 64), _n(2, 64)),
    "si_snr": (tm.audio.ScaleInvariantSignalNoiseRatio, F.audio.scale_invariant_signal_noise_ratio, _n(2, 64),
               _n(2, 64)),
    "si_sdr": (tm.audio.ScaleInvariantSignalDistortionRatio, F.audio.scale_invariant_signal_distortion_ratio,
               _n(2, 64), _n(2, 64)),
    "sa_sdr": (tm.audio.SourceAggregatedSignalDistortionRatio, F.audio.source_aggregated_signal_distortion_ratio,
               _n(1, 2, 64), _n(1, 2, 64)),
    # image
    "psnr": (partial(tm.image.PeakSignalNoiseRatio, data_range=1.0),
             partial(F.image.peak_signal_noise_ratio, data_range=1.0), _t(2, 1, 12, 12), _t(2, 1, 12, 12)),
    "ssim": (partial(tm.image.StructuralSimilarityIndexMeasure, data_range=1.0, kernel_size=5),
             partial(F.image.structural_similarity_index_measure, data_range=1.0, kernel_size=5),
             _t(2, 1, 16, 16), _t(2, 1, 16, 16)),
    "uqi": (partial(tm.image.UniversalImageQualityIndex, kernel_size=(5, 5)),
            partial(F.image.universal_image_quality_index, kernel_size=(5, 5)), _t(2, 1, 16, 16), _t(2, 1, 16, 16)),
    "sam": (tm.image.SpectralAngleMapper, F.image.spectral_angle_mapper, _t(2, 3, 8, 8) + 0.1,
            _t(2, 3, 8, 8) + 0.1),
    "ergas": (tm.image.ErrorRelativeGlobalDimensionlessSynthesis,
              F.image.error_relative_global_dimensionless_synthesis, _t(2, 3, 8, 8) + 0.1, _t(2, 3, 8, 8) + 0.1),
    "rase": (partial(tm.image.RelativeAverageSpectralError, window_size=4),
             partial(F.image.relative_average_spectral_error, window_size=4), _t(2, 3, 12, 12), _t(2, 3, 12, 12)),
    "rmse_sw": (partial(tm.image.RootMeanSquaredErrorUsingSlidingWindow, window_size=4),
                partial(F.image.root_mean_squared_error_using_sliding_window, window_size=4), _t(2, 3, 12, 12),
                _t(2, 3, 12, 12)),
    "image_gradients_tv": (tm.image.TotalVariation, None, _t(2, 3, 8, 8), None),
    # nominal / clustering (integer inputs: differentiability only through the declared flag)
    "cramers_v": (partial(tm.nominal.CramersV, num_classes=4), None, _i(4, 30), _i(4, 30)),
}


def _call(fn, preds, target):
    return fn(preds) if target is None else fn(preds, target)


@pytest.mark.parametrize("name", sorted(CASES))
def test_differentiability(name):
    factory, functional, preds, target = CASES[name]
    metric = factory()
    if not preds.is_floating_point():
        assert not metric.is_differentiable
        return
    p = preds.clone().requires_grad_(True)
    out = _call(metric, p, target)
    outs = out if isinstance(out, (tuple, list)) else [out]
    assert all(o.requires_grad == bool(metric.is_differentiable) for o in outs if torch.is_tensor(o))
    if metric.is_differentiable and functional is not None:
        tgt = target.double() if torch.is_tensor(target) and target.is_floating_point() else target
        assert torch.autograd.gradcheck(lambda x: _call(functional, x, tgt), (preds.double().requires_grad_(True),),
                                        eps=1e-6, atol=1e-4)


def _lowp(x, dtype, device):
    if x is None:
        return None
    return x.to(device=device, dtype=dtype) if x.is_floating_point() else x.to(device)


def _assert_finite_tensor(out):
    outs = out if isinstance(out, (tuple, list)) else [out]
    for o in outs:
        assert torch.is_tensor(o)


# 16-bit inputs whose reference runs are skipped on CPU (torch has no half kernels for the op on CPU)
_CPU_HALF_SKIP = {"kendall", "spearman"}


@pytest.mark.parametrize("dtype", [torch.half, torch.bfloat16])
@pytest.mark.parametrize("name", sorted(CASES))
def test_low_precision_cpu(name, dtype):
    if name in _CPU_HALF_SKIP:
        pytest.skip("no CPU 16-bit kernel in torch for this op (the reference skips it too)")
    factory, functional, preds, target = CASES[name]
    p, t = _lowp(preds, dtype, "cpu"), _lowp(target, dtype, "cpu")
    _assert_finite_tensor(_call(factory(), p, t))
    if functional is not None:
        _assert_finite_tensor(_call(functional, p, t))


_DTYPE_EPS = {"snr", "si_snr", "si_sdr", "sa_sdr"}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.half, torch.bfloat16])
@pytest.mark.parametrize("name", sorted(CASES))
def test_low_precision_gpu(name, dtype):
    """16-bit CUDA inputs go through the HIP kernels; the result must track the fp32 result of the same inputs."""
    factory, functional, preds, target = CASES[name]
    p, t = _lowp(preds, dtype, "cuda"), _lowp(target, dtype, "cuda")
    m = factory().cuda()
    low = _call(m, p, t)
    _assert_finite_tensor(low)
    ref = _call(factory().cuda(), p.float() if p.is_floating_point() else p,
                t.float() if torch.is_tensor(t) and t.is_floating_point() else t)
    lows = low if isinstance(low, (tuple, list)) else [low]
    refs = ref if isinstance(ref, (tuple, list)) else [ref]
    # the audio family adds finfo(input dtype).eps (as the reference does): bf16's eps is 7.8e-3, so its values move
    tol = 0.15 if name in _DTYPE_EPS else 0.05
    for a, b in zip(lows, refs):
        torch.testing.assert_close(a.float(), b.float(), atol=tol, rtol=tol, equal_nan=True)
    if functional is not None:
        _assert_finite_tensor(_call(functional, p, t))
