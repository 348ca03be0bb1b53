"""Feature networks used by metrics (defined natively; run on PyTorch-ROCm)."""
from torchmetrics_amd.models.inception import InceptionV3Features, NoTrainInceptionV3  # noqa: F401
