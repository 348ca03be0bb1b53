"""Functional image metrics (parity: reference ``F/image/__init__.py``)."""
from torchmetrics_amd.functional.image.basic import (
    error_relative_global_dimensionless_synthesis,
    image_gradients,
    peak_signal_noise_ratio,
    peak_signal_noise_ratio_with_blocked_effect,
    relative_average_spectral_error,
    root_mean_squared_error_using_sliding_window,
    spectral_angle_mapper,
    total_variation,
)
from torchmetrics_amd.functional.image.lpips import learned_perceptual_image_patch_similarity
from torchmetrics_amd.functional.image.perceptual_path_length import perceptual_path_length
from torchmetrics_amd.functional.image.spatial import (
    quality_with_no_reference,
    spatial_correlation_coefficient,
    spatial_distortion_index,
    spectral_distortion_index,
    visual_information_fidelity,
)
from torchmetrics_amd.functional.image.ssim import (
    multiscale_structural_similarity_index_measure,
    structural_similarity_index_measure,
    universal_image_quality_index,
)

__all__ = [k for k in dir() if not k.startswith("_")]
