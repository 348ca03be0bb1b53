"""InceptionV3 feature extractor with the FID ("pt_inception-2015-12-05") topology.

The reference wraps torch-fidelity's ``FeatureExtractorInceptionV3`` (``S/image/fid.py:44-156``), which downloads
pretrained weights.  Neither torch-fidelity nor a network are available here, so this module defines the same
architecture natively (BN-folded-friendly ``conv -> bn(eps=1e-3) -> relu`` blocks, FID-variant pooling) and runs it on
PyTorch-ROCm (MIOpen convolutions, channels-last, bf16-capable).  Weights:

* ``weights=None`` -> deterministic random init (valid for throughput benchmarks, not comparable FID values);
* ``weights="<path>"`` or env ``TORCHMETRICS_AMD_INCEPTION_WEIGHTS`` -> a ``state_dict`` saved with
  ``torch.save`` (loaded with ``weights_only=True``), in this module's parameter naming.

Feature taps match torch-fidelity's names: ``"64"``, ``"192"``, ``"768"``, ``"2048"``, ``"logits_unbiased"``,
``"1008"`` (logits).
"""
import os
from typing import Dict, List, Optional, Sequence, Tuple, Union

import torch
import torch.nn.functional as F
from torch import Tensor, nn

FID_INPUT_SIZE = 299


class BasicConv2d(nn.Module):
    def __init__(self, cin: int, cout: int, **kw: object) -> None:
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, bias=False, **kw)  # type: ignore[arg-type]
        self.bn = nn.BatchNorm2d(cout, eps=0.001)

    def forward(self, x: Tensor) -> Tensor:
        return F.relu(self.bn(self.conv(x)), inplace=True)


class InceptionA(nn.Module):
    def __init__(self, cin: int, pool_features: int) -> None:
        super().__init__()
        self.branch1x1 = BasicConv2d(cin, 64, kernel_size=1)
        self.branch5x5_1 = BasicConv2d(cin, 48, kernel_size=1)
        self.branch5x5_2 = BasicConv2d(48, 64, kernel_size=5, padding=2)
        self.branch3x3dbl_1 = BasicConv2d(cin, 64, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, kernel_size=3, padding=1)
        self.branch_pool = BasicConv2d(cin, pool_features, kernel_size=1)

    def forward(self, x: Tensor) -> Tensor:
        b1 = self.branch1x1(x)
        b5 = self.branch5x5_2(self.branch5x5_1(x))
        b3 = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x)))
        bp = self.branch_pool(F.avg_pool2d(x, kernel_size=3, stride=1, padding=1, count_include_pad=False))
        return torch.cat([b1, b5, b3, bp], 1)


class InceptionB(nn.Module):
    def __init__(self, cin: int) -> None:
        super().__init__()
        self.branch3x3 = BasicConv2d(cin, 384, kernel_size=3, stride=2)
        self.branch3x3dbl_1 = BasicConv2d(cin, 64, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, kernel_size=3, stride=2)

    def forward(self, x: Tensor) -> Tensor:
        b3 = self.branch3x3(x)
        bd = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x)))
        bp = F.max_pool2d(x, kernel_size=3, stride=2)
        return torch.cat([b3, bd, bp], 1)


class InceptionC(nn.Module):
    def __init__(self, cin: int, c7: int) -> None:
        super().__init__()
        self.branch1x1 = BasicConv2d(cin, 192, kernel_size=1)
        self.branch7x7_1 = BasicConv2d(cin, c7, kernel_size=1)
        self.branch7x7_2 = BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7_3 = BasicConv2d(c7, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_1 = BasicConv2d(cin, c7, kernel_size=1)
        self.branch7x7dbl_2 = BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_3 = BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7dbl_4 = BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_5 = BasicConv2d(c7, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch_pool = BasicConv2d(cin, 192, kernel_size=1)

    def forward(self, x: Tensor) -> Tensor:
        b1 = self.branch1x1(x)
        b7 = self.branch7x7_3(self.branch7x7_2(self.branch7x7_1(x)))
        bd = self.branch7x7dbl_1(x)
        for layer in (self.branch7x7dbl_2, self.branch7x7dbl_3, self.branch7x7dbl_4, self.branch7x7dbl_5):
            bd = layer(bd)
        bp = self.branch_pool(F.avg_pool2d(x, kernel_size=3, stride=1, padding=1, count_include_pad=False))
        return torch.cat([b1, b7, bd, bp], 1)


class InceptionD(nn.Module):
    def __init__(self, cin: int) -> None:
        super().__init__()
        self.branch3x3_1 = BasicConv2d(cin, 192, kernel_size=1)
        self.branch3x3_2 = BasicConv2d(192, 320, kernel_size=3, stride=2)
        self.branch7x7x3_1 = BasicConv2d(cin, 192, kernel_size=1)
        self.branch7x7x3_2 = BasicConv2d(192, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7x3_3 = BasicConv2d(192, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7x3_4 = BasicConv2d(192, 192, kernel_size=3, stride=2)

    def forward(self, x: Tensor) -> Tensor:
        b3 = self.branch3x3_2(self.branch3x3_1(x))
        b7 = self.branch7x7x3_4(self.branch7x7x3_3(self.branch7x7x3_2(self.branch7x7x3_1(x))))
        bp = F.max_pool2d(x, kernel_size=3, stride=2)
        return torch.cat([b3, b7, bp], 1)


class InceptionE(nn.Module):
    """``pool="avg"`` for Mixed_7b, ``pool="max"`` for Mixed_7c (the FID-graph quirk)."""

    def __init__(self, cin: int, pool: str) -> None:
        super().__init__()
        self.pool = pool
        self.branch1x1 = BasicConv2d(cin, 320, kernel_size=1)
        self.branch3x3_1 = BasicConv2d(cin, 384, kernel_size=1)
        self.branch3x3_2a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3_2b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch3x3dbl_1 = BasicConv2d(cin, 448, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(448, 384, kernel_size=3, padding=1)
        self.branch3x3dbl_3a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3dbl_3b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch_pool = BasicConv2d(cin, 192, kernel_size=1)

    def forward(self, x: Tensor) -> Tensor:
        b1 = self.branch1x1(x)
        b3 = self.branch3x3_1(x)
        b3 = torch.cat([self.branch3x3_2a(b3), self.branch3x3_2b(b3)], 1)
        bd = self.branch3x3dbl_2(self.branch3x3dbl_1(x))
        bd = torch.cat([self.branch3x3dbl_3a(bd), self.branch3x3dbl_3b(bd)], 1)
        if self.pool == "avg":
            bp = F.avg_pool2d(x, kernel_size=3, stride=1, padding=1, count_include_pad=False)
        else:
            bp = F.max_pool2d(x, kernel_size=3, stride=1, padding=1)
        bp = self.branch_pool(bp)
        return torch.cat([b1, b3, bd, bp], 1)


class InceptionV3Features(nn.Module):
    """FID InceptionV3 returning the requested feature taps (eval mode, no grad)."""

    VALID = ("64", "192", "768", "2048", "logits_unbiased", "1008")

    def __init__(self, features_list: Sequence[str] = ("2048",), weights: Optional[str] = None,
                 resize_input: bool = True) -> None:
        super().__init__()
        for f in features_list:
            if f not in self.VALID:
                raise ValueError(f"Unknown feature tap {f}; expected one of {self.VALID}")
        self.features_list = list(features_list)
        self.resize_input = resize_input
        self.Conv2d_1a_3x3 = BasicConv2d(3, 32, kernel_size=3, stride=2)
        self.Conv2d_2a_3x3 = BasicConv2d(32, 32, kernel_size=3)
        self.Conv2d_2b_3x3 = BasicConv2d(32, 64, kernel_size=3, padding=1)
        self.Conv2d_3b_1x1 = BasicConv2d(64, 80, kernel_size=1)
        self.Conv2d_4a_3x3 = BasicConv2d(80, 192, kernel_size=3)
        self.Mixed_5b = InceptionA(192, pool_features=32)
        self.Mixed_5c = InceptionA(256, pool_features=64)
        self.Mixed_5d = InceptionA(288, pool_features=64)
        self.Mixed_6a = InceptionB(288)
        self.Mixed_6b = InceptionC(768, c7=128)
        self.Mixed_6c = InceptionC(768, c7=160)
        self.Mixed_6d = InceptionC(768, c7=160)
        self.Mixed_6e = InceptionC(768, c7=192)
        self.Mixed_7a = InceptionD(768)
        self.Mixed_7b = InceptionE(1280, pool="avg")
        self.Mixed_7c = InceptionE(2048, pool="max")
        self.fc = nn.Linear(2048, 1008)
        self._init(weights)
        self.eval()
        for p in self.parameters():
            p.requires_grad_(False)

    def _init(self, weights: Optional[str]) -> None:
        path = weights or os.environ.get("TORCHMETRICS_AMD_INCEPTION_WEIGHTS")
        if path:
            self.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
            return
        g = torch.Generator().manual_seed(2015)
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                std = (2.0 / (m.weight[0].numel())) ** 0.5
                with torch.no_grad():
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * std)
                    if getattr(m, "bias", None) is not None:
                        m.bias.zero_()

    def train(self, mode: bool = True) -> "InceptionV3Features":
        return super().train(False)

    @property
    def num_features(self) -> int:
        return {"64": 64, "192": 192, "768": 768, "2048": 2048, "logits_unbiased": 1008, "1008": 1008}[
            self.features_list[-1]
        ]

    def _prep(self, x: Tensor) -> Tensor:
        if x.dtype != torch.uint8:
            raise ValueError(f"Expecting image as torch.Tensor with dtype=torch.uint8, got {x.dtype}")
        x = x.float()
        if self.resize_input and x.shape[-2:] != (FID_INPUT_SIZE, FID_INPUT_SIZE):
            x = F.interpolate(x, size=(FID_INPUT_SIZE, FID_INPUT_SIZE), mode="bilinear", align_corners=False)
        return (x - 128.0) / 128.0

    @torch.no_grad()
    def forward(self, x: Tensor) -> Union[Tensor, Tuple[Tensor, ...]]:
        want = set(self.features_list)
        out: Dict[str, Tensor] = {}
        x = self._prep(x).to(memory_format=torch.channels_last)
        x = self.Conv2d_2b_3x3(self.Conv2d_2a_3x3(self.Conv2d_1a_3x3(x)))
        x = F.max_pool2d(x, kernel_size=3, stride=2)
        if "64" in want:
            out["64"] = F.adaptive_avg_pool2d(x, 1).flatten(1)
        x = self.Conv2d_4a_3x3(self.Conv2d_3b_1x1(x))
        x = F.max_pool2d(x, kernel_size=3, stride=2)
        if "192" in want:
            out["192"] = F.adaptive_avg_pool2d(x, 1).flatten(1)
        for blk in (self.Mixed_5b, self.Mixed_5c, self.Mixed_5d, self.Mixed_6a, self.Mixed_6b, self.Mixed_6c,
                    self.Mixed_6d, self.Mixed_6e):
            x = blk(x)
        if "768" in want:
            out["768"] = F.adaptive_avg_pool2d(x, 1).flatten(1)
        x = self.Mixed_7c(self.Mixed_7b(self.Mixed_7a(x)))
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        if "2048" in want:
            out["2048"] = x
        if "logits_unbiased" in want:
            out["logits_unbiased"] = x.mm(self.fc.weight.t())
        if "1008" in want:
            out["1008"] = self.fc(x)
        res = tuple(out[f] for f in self.features_list)
        return res[0] if len(res) == 1 else res


class NoTrainInceptionV3(InceptionV3Features):
    """Reference-compatible constructor (``S/image/fid.py:44-69``): ``NoTrainInceptionV3(name, features_list,
    feature_extractor_weights_path)``; never leaves eval mode.  ``name`` is kept for API parity (the topology is
    always the FID InceptionV3); weights come from ``feature_extractor_weights_path`` or
    ``$TORCHMETRICS_AMD_INCEPTION_WEIGHTS`` (torch-fidelity's ``pt_inception-2015-12-05`` state dict layout)."""

    def __init__(self, name: str = "inception-v3-compat", features_list: Optional[Sequence[str]] = None,
                 feature_extractor_weights_path: Optional[str] = None) -> None:
        super().__init__(features_list or ["2048"], weights=feature_extractor_weights_path)
        self.name = name
