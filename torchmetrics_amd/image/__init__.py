"""Image module metrics (parity: reference ``S/image/__init__.py``)."""
from torchmetrics_amd.image.generative import (
    FrechetInceptionDistance,
    InceptionScore,
    KernelInceptionDistance,
    MemorizationInformedFrechetInceptionDistance,
)

__all__ = [k for k in dir() if k[0].isupper()]
