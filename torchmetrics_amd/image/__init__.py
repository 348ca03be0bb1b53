"""Image module metrics (parity: reference ``S/image/__init__.py``)."""
from torchmetrics_amd.image.generative import (
    FrechetInceptionDistance,
    InceptionScore,
    KernelInceptionDistance,
    MemorizationInformedFrechetInceptionDistance,
)
from torchmetrics_amd.models.inception import NoTrainInceptionV3  # noqa: F401
from torchmetrics_amd.image.perceptual import LearnedPerceptualImagePatchSimilarity, PerceptualPathLength
from torchmetrics_amd.image.quality import (
    ErrorRelativeGlobalDimensionlessSynthesis,
    MultiScaleStructuralSimilarityIndexMeasure,
    PeakSignalNoiseRatio,
    PeakSignalNoiseRatioWithBlockedEffect,
    QualityWithNoReference,
    RelativeAverageSpectralError,
    RootMeanSquaredErrorUsingSlidingWindow,
    SpatialCorrelationCoefficient,
    SpatialDistortionIndex,
    SpectralAngleMapper,
    SpectralDistortionIndex,
    StructuralSimilarityIndexMeasure,
    TotalVariation,
    UniversalImageQualityIndex,
    VisualInformationFidelity,
)

__all__ = [k for k in dir() if k[0].isupper()]
