"""Image quality module metrics (parity: reference ``S/image/{ssim,psnr,psnrb,uqi,scc,vif,rmse_sw,rase,sam,ergas,tv,
d_lambda,d_s,qnr}.py``).  State names / reductions follow the reference; SSIM, MS-SSIM and UQI updates run the fused
HIP window kernel on ROCm (see :mod:`torchmetrics_amd.functional.image.ssim`).
"""
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd.functional.image.basic import (
    _ergas_compute,
    _ergas_update,
    _psnr_compute,
    _psnr_update,
    _psnrb_compute,
    _psnrb_update,
    _rmse_sw_compute,
    _rmse_sw_update,
    _sam_compute,
    _sam_update,
    _total_variation_compute,
    _total_variation_update,
    relative_average_spectral_error,
)
from torchmetrics_amd.functional.image.spatial import (
    _scc_map,
    _scc_plane_means,
    _scc_update,
    _spatial_distortion_index_compute,
    _spatial_distortion_index_update,
    _spectral_distortion_index_compute,
    _spectral_distortion_index_update,
    _vif_planes,
)
from torchmetrics_amd.functional.image.ssim import (
    _multiscale_ssim_update,
    _ssim_check_inputs,
    _ssim_update,
    _uqi_compute,
    _uqi_update,
)
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import dim_zero_cat
from torchmetrics_amd.utilities.prints import rank_zero_warn

_Red = Literal["elementwise_mean", "sum", "none", None]


def _check_reduction(reduction: Any) -> None:
    valid = ("elementwise_mean", "sum", "none", None)
    if reduction not in valid:
        raise ValueError(f"Argument `reduction` must be one of {valid}, but got {reduction}")


class StructuralSimilarityIndexMeasure(Metric):
    """SSIM (2-D / 3-D); sums per-image scores unless ``reduction`` keeps them."""

    higher_is_better: bool = True
    is_differentiable: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        gaussian_kernel: bool = True,
        sigma: Union[float, Sequence[float]] = 1.5,
        kernel_size: Union[int, Sequence[int]] = 11,
        reduction: _Red = "elementwise_mean",
        data_range: Optional[Union[float, Tuple[float, float]]] = None,
        k1: float = 0.01,
        k2: float = 0.03,
        return_full_image: bool = False,
        return_contrast_sensitivity: bool = False,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        _check_reduction(reduction)
        if reduction in ("elementwise_mean", "sum"):
            self.add_state("similarity", default=torch.tensor(0.0), dist_reduce_fx="sum")
        else:
            self.add_state("similarity", default=[], dist_reduce_fx="cat")
        self.add_state("total", default=torch.tensor(0.0), dist_reduce_fx="sum")
        if return_contrast_sensitivity or return_full_image:
            self.add_state("image_return", default=[], dist_reduce_fx="cat")
        self.gaussian_kernel = gaussian_kernel
        self.sigma = sigma
        self.kernel_size = kernel_size
        self.reduction = reduction
        self.data_range = data_range
        self.k1 = k1
        self.k2 = k2
        self.return_full_image = return_full_image
        self.return_contrast_sensitivity = return_contrast_sensitivity

    def update(self, preds: Tensor, target: Tensor) -> None:
        preds, target = _ssim_check_inputs(preds, target)
        pack = _ssim_update(preds, target, self.gaussian_kernel, self.sigma, self.kernel_size, self.data_range,
                            self.k1, self.k2, self.return_full_image, self.return_contrast_sensitivity)
        similarity, image = pack if isinstance(pack, tuple) else (pack, None)
        if image is not None:
            self.image_return.append(image)
        if self.reduction in ("elementwise_mean", "sum"):
            self.similarity += similarity.sum()
            self.total += preds.shape[0]
        else:
            self.similarity.append(similarity)

    def compute(self) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        if self.reduction == "elementwise_mean":
            similarity = self.similarity / self.total
        elif self.reduction == "sum":
            similarity = self.similarity
        else:
            similarity = dim_zero_cat(self.similarity)
        if self.return_contrast_sensitivity or self.return_full_image:
            return similarity, dim_zero_cat(self.image_return)
        return similarity


class MultiScaleStructuralSimilarityIndexMeasure(Metric):
    """MS-SSIM over ``len(betas)`` dyadic scales."""

    higher_is_better: bool = True
    is_differentiable: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        gaussian_kernel: bool = True,
        kernel_size: Union[int, Sequence[int]] = 11,
        sigma: Union[float, Sequence[float]] = 1.5,
        reduction: _Red = "elementwise_mean",
        data_range: Optional[Union[float, Tuple[float, float]]] = None,
        k1: float = 0.01,
        k2: float = 0.03,
        betas: Tuple[float, ...] = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333),
        normalize: Literal["relu", "simple", None] = "relu",
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        _check_reduction(reduction)
        if reduction in ("elementwise_mean", "sum"):
            self.add_state("similarity", default=torch.tensor(0.0), dist_reduce_fx="sum")
        else:
            self.add_state("similarity", default=[], dist_reduce_fx="cat")
        self.add_state("total", default=torch.tensor(0.0), dist_reduce_fx="sum")
        if not isinstance(kernel_size, (Sequence, int)):
            raise ValueError(
                f"Argument `kernel_size` expected to be an sequence or an int, or a single int. Got {kernel_size}"
            )
        if isinstance(kernel_size, Sequence) and (
            len(kernel_size) not in (2, 3) or not all(isinstance(ks, int) for ks in kernel_size)
        ):
            raise ValueError(
                "Argument `kernel_size` expected to be an sequence of size 2 or 3 where each element is an int, "
                f"or a single int. Got {kernel_size}"
            )
        if not isinstance(betas, tuple):
            raise ValueError("Argument `betas` is expected to be of a type tuple.")
        if not all(isinstance(beta, float) for beta in betas):
            raise ValueError("Argument `betas` is expected to be a tuple of floats.")
        if normalize and normalize not in ("relu", "simple"):
            raise ValueError("Argument `normalize` to be expected either `None` or one of 'relu' or 'simple'")
        self.gaussian_kernel = gaussian_kernel
        self.sigma = sigma
        self.kernel_size = kernel_size
        self.reduction = reduction
        self.data_range = data_range
        self.k1 = k1
        self.k2 = k2
        self.betas = betas
        self.normalize = normalize

    def update(self, preds: Tensor, target: Tensor) -> None:
        preds, target = _ssim_check_inputs(preds, target)
        sim = _multiscale_ssim_update(preds, target, self.gaussian_kernel, self.sigma, self.kernel_size,
                                      self.data_range, self.k1, self.k2, self.betas, self.normalize)
        if self.reduction in ("none", None):
            self.similarity.append(sim)
        else:
            self.similarity += sim.sum()
        self.total += preds.shape[0]

    def compute(self) -> Tensor:
        if self.reduction in ("none", None):
            return dim_zero_cat(self.similarity)
        if self.reduction == "sum":
            return self.similarity
        return self.similarity / self.total


class PeakSignalNoiseRatio(Metric):
    """PSNR; with ``data_range=None`` the range is tracked from the target min / max across updates."""

    is_differentiable: bool = True
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0

    def __init__(
        self,
        data_range: Optional[Union[float, Tuple[float, float]]] = None,
        base: float = 10.0,
        reduction: _Red = "elementwise_mean",
        dim: Optional[Union[int, Tuple[int, ...]]] = None,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if dim is None and reduction != "elementwise_mean":
            rank_zero_warn(f"The `reduction={reduction}` will not have any effect when `dim` is None.")
        if dim is None:
            self.add_state("sum_squared_error", default=torch.tensor(0.0), dist_reduce_fx="sum")
            self.add_state("total", default=torch.tensor(0), dist_reduce_fx="sum")
        else:
            self.add_state("sum_squared_error", default=[], dist_reduce_fx="cat")
            self.add_state("total", default=[], dist_reduce_fx="cat")
        self.clamp_range = None
        if data_range is None:
            if dim is not None:
                raise ValueError("The `data_range` must be given when `dim` is not None.")
            self.data_range = None
            self.add_state("min_target", default=torch.tensor(0.0), dist_reduce_fx=torch.min)
            self.add_state("max_target", default=torch.tensor(0.0), dist_reduce_fx=torch.max)
        elif isinstance(data_range, tuple):
            self.add_state("data_range", default=torch.tensor(data_range[1] - data_range[0]), dist_reduce_fx="mean")
            self.clamp_range = data_range
        else:
            self.add_state("data_range", default=torch.tensor(float(data_range)), dist_reduce_fx="mean")
        self.base = base
        self.reduction = reduction
        self.dim = tuple(dim) if isinstance(dim, Sequence) else dim

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.clamp_range is not None:
            preds = preds.clamp(*self.clamp_range)
            target = target.clamp(*self.clamp_range)
        sse, num_obs = _psnr_update(preds, target, dim=self.dim)
        if self.dim is None:
            if self.data_range is None:
                self.min_target = torch.minimum(target.min(), self.min_target)
                self.max_target = torch.maximum(target.max(), self.max_target)
            self.sum_squared_error += sse
            self.total += num_obs
        else:
            self.sum_squared_error.append(sse)
            self.total.append(num_obs)

    def compute(self) -> Tensor:
        data_range = self.data_range if self.data_range is not None else self.max_target - self.min_target
        if self.dim is None:
            sse, total = self.sum_squared_error, self.total
        else:
            sse = torch.cat([v.flatten() for v in self.sum_squared_error])
            total = torch.cat([v.flatten() for v in self.total])
        return _psnr_compute(sse, total, data_range, base=self.base, reduction=self.reduction)


class PeakSignalNoiseRatioWithBlockedEffect(Metric):
    """PSNR-B for grayscale images (blocking-effect corrected)."""

    is_differentiable: bool = True
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: Optional[float] = None

    def __init__(self, block_size: int = 8, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not isinstance(block_size, int) and block_size < 1:
            raise ValueError("Argument ``block_size`` should be a positive integer")
        self.block_size = block_size
        self.add_state("sum_squared_error", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", default=torch.tensor(0), dist_reduce_fx="sum")
        self.add_state("bef", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("data_range", default=torch.tensor(0), dist_reduce_fx="max")

    def update(self, preds: Tensor, target: Tensor) -> None:
        sse, bef, num_obs = _psnrb_update(preds, target, block_size=self.block_size)
        self.sum_squared_error += sse
        self.bef += bef
        self.total += num_obs
        self.data_range = torch.maximum(self.data_range, torch.max(target) - torch.min(target))

    def compute(self) -> Tensor:
        return _psnrb_compute(self.sum_squared_error, self.bef, self.total, self.data_range)


class UniversalImageQualityIndex(Metric):
    """UQI; mean / sum reductions accumulate in-kernel partial sums, ``none`` keeps the images."""

    is_differentiable: bool = True
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, kernel_size: Sequence[int] = (11, 11), sigma: Sequence[float] = (1.5, 1.5),
                 reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean",
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if reduction is None or reduction == "none":
            self.add_state("preds", default=[], dist_reduce_fx="cat")
            self.add_state("target", default=[], dist_reduce_fx="cat")
        else:
            self.add_state("sum_uqi", torch.tensor(0.0), dist_reduce_fx="sum")
            self.add_state("numel", torch.tensor(0), dist_reduce_fx="sum")
        self.kernel_size = kernel_size
        self.sigma = sigma
        self.reduction = reduction

    def update(self, preds: Tensor, target: Tensor) -> None:
        preds, target = _uqi_update(preds, target)
        if self.reduction is None or self.reduction == "none":
            self.preds.append(preds)
            self.target.append(target)
        else:
            self.sum_uqi += _uqi_compute(preds, target, self.kernel_size, self.sigma, reduction="sum")
            b, c, h, w = preds.shape
            self.numel += b * c * (h - self.kernel_size[0] + 1) * (w - self.kernel_size[1] + 1)

    def compute(self) -> Tensor:
        if self.reduction is None or self.reduction == "none":
            return _uqi_compute(dim_zero_cat(self.preds), dim_zero_cat(self.target), self.kernel_size, self.sigma,
                                self.reduction)
        return self.sum_uqi / self.numel if self.reduction == "elementwise_mean" else self.sum_uqi


class SpatialCorrelationCoefficient(Metric):
    """Spatial correlation coefficient of Laplacian high-pass images."""

    is_differentiable = True
    higher_is_better = True
    full_state_update = False
    plot_lower_bound: Optional[float] = None
    plot_upper_bound: Optional[float] = None

    def __init__(self, high_pass_filter: Optional[Tensor] = None, window_size: int = 8, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if high_pass_filter is None:
            high_pass_filter = torch.tensor([[-1, -1, -1], [-1, 8, -1], [-1, -1, -1]])
        self.hp_filter = high_pass_filter
        self.ws = window_size
        self.add_state("scc_score", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", default=torch.tensor(0.0), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        preds, target, hp = _scc_update(preds, target, self.hp_filter, self.ws)
        self.scc_score += _scc_plane_means(preds, target, hp, self.ws).sum()
        self.total += preds.size(0)

    def compute(self) -> Tensor:
        return self.scc_score / self.total


class VisualInformationFidelity(Metric):
    """Pixel-domain VIF (mean over channels, then over images)."""

    is_differentiable = True
    higher_is_better = True
    full_state_update = False
    plot_lower_bound: Optional[float] = None

    def __init__(self, sigma_n_sq: float = 2.0, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not isinstance(sigma_n_sq, float) and not isinstance(sigma_n_sq, int):
            raise ValueError(f"Argument `sigma_n_sq` is expected to be a positive float or int, but got {sigma_n_sq}")
        if sigma_n_sq < 0:
            raise ValueError(f"Argument `sigma_n_sq` is expected to be a positive float or int, but got {sigma_n_sq}")
        self.add_state("vif_score", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.sigma_n_sq = sigma_n_sq

    def update(self, preds: Tensor, target: Tensor) -> None:
        b, c, h, w = preds.shape
        planes_p = preds.transpose(0, 1).reshape(c * b, 1, h, w)
        planes_t = target.transpose(0, 1).reshape(c * b, 1, h, w)
        per_image = _vif_planes(planes_p, planes_t, self.sigma_n_sq).reshape(c, b).mean(0)
        self.vif_score += per_image.sum()
        self.total += b

    def compute(self) -> Tensor:
        return self.vif_score / self.total


class RootMeanSquaredErrorUsingSlidingWindow(Metric):
    """RMSE over sliding windows."""

    higher_is_better: bool = False
    is_differentiable: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0

    def __init__(self, window_size: int = 8, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not isinstance(window_size, int) or window_size < 1:
            raise ValueError("Argument `window_size` is expected to be a positive integer.")
        self.window_size = window_size
        self.add_state("rmse_val_sum", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total_images", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.rmse_map: Optional[Tensor] = None

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self.rmse_map is None:
            self.rmse_map = torch.zeros(target.shape[1:], dtype=target.dtype, device=target.device)
        self.rmse_val_sum, self.rmse_map, self.total_images = _rmse_sw_update(
            preds, target, self.window_size, self.rmse_val_sum, self.rmse_map, self.total_images
        )

    def compute(self) -> Optional[Tensor]:
        rmse, _ = _rmse_sw_compute(self.rmse_val_sum, self.rmse_map, self.total_images)
        return rmse


class RelativeAverageSpectralError(Metric):
    """RASE over all accumulated images."""

    higher_is_better: bool = False
    is_differentiable: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0

    def __init__(self, window_size: int = 8, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not isinstance(window_size, int) or window_size < 1:
            raise ValueError(f"Argument `window_size` is expected to be a positive integer, but got {window_size}")
        self.window_size = window_size
        self.add_state("preds", default=[], dist_reduce_fx="cat")
        self.add_state("target", default=[], dist_reduce_fx="cat")
        rank_zero_warn(
            "Metric `RelativeAverageSpectralError` will save all targets and predictions in the buffer."
            " For large datasets, this may lead to large memory footprint."
        )

    def update(self, preds: Tensor, target: Tensor) -> None:
        self.preds.append(preds)
        self.target.append(target)

    def compute(self) -> Tensor:
        return relative_average_spectral_error(dim_zero_cat(self.preds), dim_zero_cat(self.target), self.window_size)


class SpectralAngleMapper(Metric):
    """Spectral angle mapper (radians)."""

    plot_upper_bound: Optional[float] = 1.0
    higher_is_better: bool = False
    is_differentiable: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0

    def __init__(self, reduction: _Red = "elementwise_mean", **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if reduction in ("none", None):
            rank_zero_warn(
                "Metric `SpectralAngleMapper` will save all targets and predictions in the buffer when using"
                "`reduction=None` or `reduction='none'. For large datasets, this may lead to a large memory footprint."
            )
            self.add_state("preds", default=[], dist_reduce_fx="cat")
            self.add_state("target", default=[], dist_reduce_fx="cat")
        else:
            self.add_state("sum_sam", torch.tensor(0.0), dist_reduce_fx="sum")
            self.add_state("numel", torch.tensor(0), dist_reduce_fx="sum")
        self.reduction = reduction

    def update(self, preds: Tensor, target: Tensor) -> None:
        preds, target = _sam_update(preds, target)
        if self.reduction in ("none", None):
            self.preds.append(preds)
            self.target.append(target)
        else:
            self.sum_sam += _sam_compute(preds, target, reduction="sum")
            self.numel += preds.shape[0] * preds.shape[2] * preds.shape[3]

    def compute(self) -> Tensor:
        if self.reduction in ("none", None):
            return _sam_compute(dim_zero_cat(self.preds), dim_zero_cat(self.target), self.reduction)
        return self.sum_sam / self.numel if self.reduction == "elementwise_mean" else self.sum_sam


class ErrorRelativeGlobalDimensionlessSynthesis(Metric):
    """ERGAS over all accumulated images."""

    higher_is_better: bool = False
    is_differentiable: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0

    def __init__(self, ratio: float = 4, reduction: _Red = "elementwise_mean", **kwargs: Any) -> None:
        super().__init__(**kwargs)
        rank_zero_warn(
            "Metric `ErrorRelativeGlobalDimensionlessSynthesis` will save all targets and"
            " predictions in buffer. For large datasets this may lead"
            " to large memory footprint."
        )
        self.add_state("preds", default=[], dist_reduce_fx="cat")
        self.add_state("target", default=[], dist_reduce_fx="cat")
        self.ratio = ratio
        self.reduction = reduction

    def update(self, preds: Tensor, target: Tensor) -> None:
        preds, target = _ergas_update(preds, target)
        self.preds.append(preds)
        self.target.append(target)

    def compute(self) -> Tensor:
        return _ergas_compute(dim_zero_cat(self.preds), dim_zero_cat(self.target), self.ratio, self.reduction)


class TotalVariation(Metric):
    """Total variation of images (``update(img)``)."""

    is_differentiable: bool = True
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0

    def __init__(self, reduction: Optional[Literal["mean", "sum", "none"]] = "sum", **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if reduction is not None and reduction not in ("sum", "mean", "none"):
            raise ValueError("Expected argument `reduction` to either be 'sum', 'mean', 'none' or None")
        self.reduction = reduction
        self.add_state("score_list", default=[], dist_reduce_fx="cat")
        self.add_state("score", default=torch.tensor(0, dtype=torch.float), dist_reduce_fx="sum")
        self.add_state("num_elements", default=torch.tensor(0, dtype=torch.int), dist_reduce_fx="sum")

    def update(self, img: Tensor) -> None:
        score, n = _total_variation_update(img)
        if self.reduction is None or self.reduction == "none":
            self.score_list.append(score)
        else:
            self.score += score.sum()
        self.num_elements += n

    def compute(self) -> Tensor:
        score = dim_zero_cat(self.score_list) if self.reduction is None or self.reduction == "none" else self.score
        return _total_variation_compute(score, self.num_elements, self.reduction)


class SpectralDistortionIndex(Metric):
    """D_lambda between a fused image and the low-resolution multispectral image."""

    higher_is_better: bool = True
    is_differentiable: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, p: int = 1, reduction: Literal["elementwise_mean", "sum", "none"] = "elementwise_mean",
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        rank_zero_warn(
            "Metric `SpectralDistortionIndex` will save all targets and"
            " predictions in buffer. For large datasets this may lead"
            " to large memory footprint."
        )
        if not isinstance(p, int) or p <= 0:
            raise ValueError(f"Expected `p` to be a positive integer. Got p: {p}.")
        self.p = p
        allowed = ("elementwise_mean", "sum", "none")
        if reduction not in allowed:
            raise ValueError(f"Expected argument `reduction` be one of {allowed} but got {reduction}")
        self.reduction = reduction
        self.add_state("preds", default=[], dist_reduce_fx="cat")
        self.add_state("target", default=[], dist_reduce_fx="cat")

    def update(self, preds: Tensor, target: Tensor) -> None:
        preds, target = _spectral_distortion_index_update(preds, target)
        self.preds.append(preds)
        self.target.append(target)

    def compute(self) -> Tensor:
        return _spectral_distortion_index_compute(dim_zero_cat(self.preds), dim_zero_cat(self.target), self.p,
                                                  self.reduction)


class _PansharpenBase(Metric):
    higher_is_better: bool = True
    is_differentiable: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def _init_states(self) -> None:
        for name in ("preds", "ms", "pan", "pan_lr"):
            self.add_state(name, default=[], dist_reduce_fx="cat")

    def update(self, preds: Tensor, target: Dict[str, Tensor]) -> None:
        if "ms" not in target:
            raise ValueError(f"Expected `target` to have key `ms`. Got target: {target.keys()}.")
        if "pan" not in target:
            raise ValueError(f"Expected `target` to have key `pan`. Got target: {target.keys()}.")
        _spatial_distortion_index_update(preds, target["ms"], target["pan"], target.get("pan_lr"))
        self.preds.append(preds)
        self.ms.append(target["ms"])
        self.pan.append(target["pan"])
        if "pan_lr" in target:
            self.pan_lr.append(target["pan_lr"])

    def _cat(self) -> Tuple[Tensor, Tensor, Tensor, Optional[Tensor]]:
        pan_lr = dim_zero_cat(self.pan_lr) if len(self.pan_lr) > 0 else None
        return dim_zero_cat(self.preds), dim_zero_cat(self.ms), dim_zero_cat(self.pan), pan_lr


def _check_pansharpen_args(norm_order: int, window_size: int, reduction: str) -> None:
    if not isinstance(norm_order, int) or norm_order <= 0:
        raise ValueError(f"Expected `norm_order` to be a positive integer. Got norm_order: {norm_order}.")
    if not isinstance(window_size, int) or window_size <= 0:
        raise ValueError(f"Expected `window_size` to be a positive integer. Got window_size: {window_size}.")
    allowed = ("elementwise_mean", "sum", "none")
    if reduction not in allowed:
        raise ValueError(f"Expected argument `reduction` be one of {allowed} but got {reduction}")


class SpatialDistortionIndex(_PansharpenBase):
    """D_s: spatial distortion index (``update(preds, {"ms", "pan"[, "pan_lr"]})``)."""

    def __init__(self, norm_order: int = 1, window_size: int = 7,
                 reduction: Literal["elementwise_mean", "sum", "none"] = "elementwise_mean", **kwargs: Any) -> None:
        super().__init__(**kwargs)
        rank_zero_warn(
            "Metric `SpatialDistortionIndex` will save all targets and"
            " predictions in buffer. For large datasets this may lead"
            " to large memory footprint."
        )
        _check_pansharpen_args(norm_order, window_size, reduction)
        self.norm_order = norm_order
        self.window_size = window_size
        self.reduction = reduction
        self._init_states()

    def compute(self) -> Tensor:
        preds, ms, pan, pan_lr = self._cat()
        return _spatial_distortion_index_compute(preds, ms, pan, pan_lr, self.norm_order, self.window_size,
                                                 self.reduction)


class QualityWithNoReference(_PansharpenBase):
    """QNR = (1 - D_lambda)^alpha (1 - D_s)^beta."""

    def __init__(self, alpha: float = 1, beta: float = 1, norm_order: int = 1, window_size: int = 7,
                 reduction: Literal["elementwise_mean", "sum", "none"] = "elementwise_mean", **kwargs: Any) -> None:
        super().__init__(**kwargs)
        rank_zero_warn(
            "Metric `QualityWithNoReference` will save all targets and"
            " predictions in buffer. For large datasets this may lead"
            " to large memory footprint."
        )
        if not isinstance(alpha, (int, float)) or alpha < 0:
            raise ValueError(f"Expected `alpha` to be a non-negative real number. Got alpha: {alpha}.")
        if not isinstance(beta, (int, float)) or beta < 0:
            raise ValueError(f"Expected `beta` to be a non-negative real number. Got beta: {beta}.")
        _check_pansharpen_args(norm_order, window_size, reduction)
        self.alpha = alpha
        self.beta = beta
        self.norm_order = norm_order
        self.window_size = window_size
        self.reduction = reduction
        self._init_states()

    def compute(self) -> Tensor:
        preds, ms, pan, pan_lr = self._cat()
        d_lambda = _spectral_distortion_index_compute(preds, ms, self.norm_order, self.reduction)
        d_s = _spatial_distortion_index_compute(preds, ms, pan, pan_lr, self.norm_order, self.window_size,
                                                self.reduction)
        return (1 - d_lambda) ** self.alpha * (1 - d_s) ** self.beta
