"""Audio metrics, functional API (reference ``F/audio/__init__.py``)."""
from torchmetrics_amd.functional.audio.external import perceptual_evaluation_speech_quality
from torchmetrics_amd.functional.audio.stoi import short_time_objective_intelligibility
from torchmetrics_amd.functional.audio.pit import permutation_invariant_training, pit_permutate
from torchmetrics_amd.functional.audio.srmr import speech_reverberation_modulation_energy_ratio
from torchmetrics_amd.functional.audio.snr_sdr import (
    complex_scale_invariant_signal_noise_ratio,
    scale_invariant_signal_distortion_ratio,
    scale_invariant_signal_noise_ratio,
    signal_distortion_ratio,
    signal_noise_ratio,
    source_aggregated_signal_distortion_ratio,
)

__all__ = [
    "complex_scale_invariant_signal_noise_ratio",
    "perceptual_evaluation_speech_quality",
    "permutation_invariant_training",
    "pit_permutate",
    "scale_invariant_signal_distortion_ratio",
    "scale_invariant_signal_noise_ratio",
    "short_time_objective_intelligibility",
    "signal_distortion_ratio",
    "signal_noise_ratio",
    "source_aggregated_signal_distortion_ratio",
    "speech_reverberation_modulation_energy_ratio",
]
