"""Learned Perceptual Image Patch Similarity (reference ``F/image/lpips.py``).

Backbones (AlexNet / VGG16 / SqueezeNet-1.1 feature stacks, torchvision layer layout so torchvision ImageNet
checkpoints load unchanged) run on MIOpen convolutions; the per-layer LPIPS distance -- channel-normalise both
feature maps, squared difference, learned 1x1 weighting, spatial mean -- is ONE fused HIP pass per layer
(:func:`torchmetrics_amd.ops.lpips_layer`) instead of ~6 elementwise/reduction passes.  When gradients are required
(LPIPS as a training loss) the differentiable composite path is used.

Weights are never downloaded.  ``pretrained=True`` loads the LPIPS linear heads from ``weights_path`` (or
``$TORCHMETRICS_AMD_LPIPS_DIR/{net}.pth``, or ``~/.cache/torchmetrics_amd/lpips/{net}.pth``) and the backbone from
``backbone_weights_path`` or the torch hub cache (torchvision file names); all with ``torch.load(weights_only=True)``.
"""
import os
from typing import Any, List, Literal, NamedTuple, Optional, Tuple, Union

import torch
from torch import Tensor, nn

from torchmetrics_amd import ops

_CHANNELS = {"alex": [64, 192, 384, 256, 256], "vgg": [64, 128, 256, 512, 512],
             "squeeze": [64, 128, 256, 384, 384, 512, 512]}
_SLICES = {"alex": [(0, 2), (2, 5), (5, 8), (8, 10), (10, 12)],
           "vgg": [(0, 4), (4, 9), (9, 16), (16, 23), (23, 30)],
           "squeeze": [(0, 2), (2, 5), (5, 8), (8, 10), (10, 11), (11, 12), (12, 13)]}
_HUB_FILES = {"alex": "alexnet-owt-7be5be79.pth", "vgg": "vgg16-397923af.pth", "squeeze": "squeezenet1_1-b8a52dc0.pth"}


class _Fire(nn.Module):
    """SqueezeNet fire module: 1x1 squeeze, then concatenated 1x1 / 3x3 expands."""

    def __init__(self, inplanes: int, squeeze: int, e1: int, e3: int) -> None:
        super().__init__()
        self.squeeze = nn.Conv2d(inplanes, squeeze, 1)
        self.squeeze_activation = nn.ReLU(inplace=True)
        self.expand1x1 = nn.Conv2d(squeeze, e1, 1)
        self.expand1x1_activation = nn.ReLU(inplace=True)
        self.expand3x3 = nn.Conv2d(squeeze, e3, 3, padding=1)
        self.expand3x3_activation = nn.ReLU(inplace=True)

    def forward(self, x: Tensor) -> Tensor:
        x = self.squeeze_activation(self.squeeze(x))
        return torch.cat([self.expand1x1_activation(self.expand1x1(x)),
                          self.expand3x3_activation(self.expand3x3(x))], 1)


def _features(net: str) -> List[nn.Module]:
    relu = lambda: nn.ReLU(inplace=True)  # noqa: E731
    if net == "alex":
        return [nn.Conv2d(3, 64, 11, 4, 2), relu(), nn.MaxPool2d(3, 2), nn.Conv2d(64, 192, 5, padding=2), relu(),
                nn.MaxPool2d(3, 2), nn.Conv2d(192, 384, 3, padding=1), relu(), nn.Conv2d(384, 256, 3, padding=1),
                relu(), nn.Conv2d(256, 256, 3, padding=1), relu(), nn.MaxPool2d(3, 2)]
    if net == "vgg":
        layers: List[nn.Module] = []
        cin = 3
        for v in [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
            else:
                layers += [nn.Conv2d(cin, v, 3, padding=1), relu()]
                cin = v
        return layers
    pool = lambda: nn.MaxPool2d(3, 2, ceil_mode=True)  # noqa: E731
    return [nn.Conv2d(3, 64, 3, 2), relu(), pool(), _Fire(64, 16, 64, 64), _Fire(128, 16, 64, 64), pool(),
            _Fire(128, 32, 128, 128), _Fire(256, 32, 128, 128), pool(), _Fire(256, 48, 192, 192),
            _Fire(384, 48, 192, 192), _Fire(384, 64, 256, 256), _Fire(512, 64, 256, 256)]


class _Backbone(nn.Module):
    """Feature stack split into the LPIPS taps; parameters live under ``slice{k}.{torchvision index}``."""

    def __init__(self, net: str) -> None:
        super().__init__()
        feats = _features(net)
        self.n_slices = len(_SLICES[net])
        for k, (a, b) in enumerate(_SLICES[net], start=1):
            seq = nn.Sequential()
            for i in range(a, b):
                seq.add_module(str(i), feats[i])
            setattr(self, f"slice{k}", seq)

    def forward(self, x: Tensor) -> List[Tensor]:
        outs = []
        for k in range(1, self.n_slices + 1):
            x = getattr(self, f"slice{k}")(x)
            outs.append(x)
        return outs

    def load_torchvision(self, state: dict) -> None:
        """Load a torchvision ``features.{i}.*`` checkpoint into the sliced layout."""
        index_to_slice = {}
        for k in range(1, self.n_slices + 1):
            for name in getattr(self, f"slice{k}")._modules:
                index_to_slice[name] = k
        mapped = {}
        for key, val in state.items():
            if not key.startswith("features."):
                continue
            idx, rest = key[len("features."):].split(".", 1)
            mapped[f"slice{index_to_slice[idx]}.{idx}.{rest}"] = val
        self.load_state_dict(mapped, strict=True)


class _NetLinLayer(nn.Module):
    def __init__(self, chn_in: int, use_dropout: bool = False) -> None:
        super().__init__()
        layers: List[nn.Module] = [nn.Dropout()] if use_dropout else []
        layers.append(nn.Conv2d(chn_in, 1, 1, stride=1, padding=0, bias=False))
        self.model = nn.Sequential(*layers)

    def forward(self, x: Tensor) -> Tensor:
        return self.model(x)


# ------------------------------------------------------------------------------------ public building blocks
# Same names / constructor signatures / NamedTuple outputs as the reference's torchvision-backed classes
# (F/image/lpips.py:65-255); here they are views of our own sliced backbones, with ImageNet weights read from the
# local torch-hub cache when ``pretrained=True`` (nothing is downloaded).
class _SqueezeOutput(NamedTuple):
    relu1: Tensor
    relu2: Tensor
    relu3: Tensor
    relu4: Tensor
    relu5: Tensor
    relu6: Tensor
    relu7: Tensor


class _AlexnetOutputs(NamedTuple):
    relu1: Tensor
    relu2: Tensor
    relu3: Tensor
    relu4: Tensor
    relu5: Tensor


class _VGGOutputs(NamedTuple):
    relu1_2: Tensor
    relu2_2: Tensor
    relu3_3: Tensor
    relu4_3: Tensor
    relu5_3: Tensor


class _PublicBackbone(_Backbone):
    _net = "alex"
    _out: Any = _AlexnetOutputs

    def __init__(self, requires_grad: bool = False, pretrained: bool = True) -> None:
        super().__init__(self._net)
        if pretrained:
            hub = os.path.join(torch.hub.get_dir(), "checkpoints", _HUB_FILES[self._net])
            if not os.path.isfile(hub):
                raise FileNotFoundError(f"ImageNet weights for `{self._net}` not found at {hub}; nothing is downloaded."
                                        " Use `pretrained=False` for random weights.")
            self.load_torchvision(torch.load(hub, map_location="cpu", weights_only=True))
        if not requires_grad:
            for p in self.parameters():
                p.requires_grad = False

    def forward(self, x: Tensor) -> NamedTuple:  # type: ignore[override]
        return self._out(*super().forward(x))


class SqueezeNet(_PublicBackbone):
    """SqueezeNet 1.1 feature taps (7 ReLU outputs)."""

    _net = "squeeze"
    _out = _SqueezeOutput


class Alexnet(_PublicBackbone):
    """AlexNet feature taps (5 ReLU outputs)."""

    _net = "alex"
    _out = _AlexnetOutputs


class Vgg16(_PublicBackbone):
    """VGG16 feature taps (relu1_2 ... relu5_3)."""

    _net = "vgg"
    _out = _VGGOutputs


class ScalingLayer(nn.Module):
    """LPIPS input normalisation ``(x - shift) / scale``."""

    def __init__(self) -> None:
        super().__init__()
        self.register_buffer("shift", torch.tensor([-0.030, -0.088, -0.188])[None, :, None, None], persistent=False)
        self.register_buffer("scale", torch.tensor([0.458, 0.448, 0.450])[None, :, None, None], persistent=False)

    def forward(self, inp: Tensor) -> Tensor:
        return (inp - self.shift) / self.scale


class NetLinLayer(nn.Module):
    """A single 1x1 convolution (optionally after dropout): the LPIPS per-tap channel weighting."""

    def __init__(self, chn_in: int, chn_out: int = 1, use_dropout: bool = False) -> None:
        super().__init__()
        layers: List[nn.Module] = [nn.Dropout()] if use_dropout else []
        layers.append(nn.Conv2d(chn_in, chn_out, 1, stride=1, padding=0, bias=False))
        self.model = nn.Sequential(*layers)

    def forward(self, x: Tensor) -> Tensor:
        return self.model(x)


def _find_file(explicit: Optional[str], candidates: List[str]) -> Optional[str]:
    for p in ([explicit] if explicit else []) + candidates:
        if p and os.path.isfile(p):
            return p
    return None


class _LPIPS(nn.Module):
    """LPIPS network: input scaling, backbone taps, per-tap learned channel weights."""

    def __init__(self, pretrained: bool = True, net: Literal["alex", "vgg", "squeeze"] = "alex", spatial: bool = False,
                 pnet_rand: bool = False, pnet_tune: bool = False, use_dropout: bool = True,
                 model_path: Optional[str] = None, eval_mode: bool = True, resize: Optional[int] = None,
                 backbone_weights_path: Optional[str] = None) -> None:
        super().__init__()
        net = "vgg" if net == "vgg16" else net
        if net not in _CHANNELS:
            raise ValueError(f"Argument `net_type` must be one of ('vgg', 'alex', 'squeeze'), but got {net}.")
        self.pnet_type, self.pnet_tune, self.pnet_rand, self.spatial, self.resize = net, pnet_tune, pnet_rand, spatial, resize
        self.register_buffer("shift", torch.tensor([-0.030, -0.088, -0.188])[None, :, None, None], persistent=False)
        self.register_buffer("scale", torch.tensor([0.458, 0.448, 0.450])[None, :, None, None], persistent=False)
        self.chns = _CHANNELS[net]
        self.net = _Backbone(net)
        for k, c in enumerate(self.chns):
            setattr(self, f"lin{k}", _NetLinLayer(c, use_dropout=use_dropout))
        self.lins = nn.ModuleList([getattr(self, f"lin{k}") for k in range(len(self.chns))])
        if not pnet_rand:
            hub = os.path.join(torch.hub.get_dir(), "checkpoints", _HUB_FILES[net])
            path = _find_file(backbone_weights_path, [hub])
            if path is None:
                raise FileNotFoundError(
                    f"LPIPS `{net}` backbone needs ImageNet weights (torchvision format, e.g. {hub}); none found and"
                    " nothing is downloaded. Pass `backbone_weights_path=` or use random backbone weights explicitly.")
            self.net.load_torchvision(torch.load(path, map_location="cpu", weights_only=True))
        if pretrained:
            env = os.environ.get("TORCHMETRICS_AMD_LPIPS_DIR", "")
            path = _find_file(model_path, [os.path.join(env, f"{net}.pth") if env else "",
                                           os.path.expanduser(f"~/.cache/torchmetrics_amd/lpips/{net}.pth")])
            if path is None:
                raise FileNotFoundError(
                    f"LPIPS linear-head weights for `{net}` not found (looked at `model_path`, $TORCHMETRICS_AMD_LPIPS_DIR,"
                    " ~/.cache/torchmetrics_amd/lpips); nothing is downloaded. Pass `pretrained=False` for random heads.")
            self.load_state_dict(torch.load(path, map_location="cpu", weights_only=True), strict=False)
        if eval_mode:
            self.eval()
        if not pnet_tune:
            for p in self.parameters():
                p.requires_grad = False

    def _lin_weight(self, k: int) -> Tensor:
        return self.lins[k].model[-1].weight.reshape(-1)

    def forward(self, in0: Tensor, in1: Tensor, retperlayer: bool = False,
                normalize: bool = False) -> Union[Tensor, Tuple[Tensor, List[Tensor]]]:
        if normalize:
            in0, in1 = 2 * in0 - 1, 2 * in1 - 1
        x0, x1 = (in0 - self.shift) / self.scale, (in1 - self.shift) / self.scale
        if self.resize is not None:
            x0 = nn.functional.interpolate(x0, size=(self.resize, self.resize), mode="bilinear", align_corners=False)
            x1 = nn.functional.interpolate(x1, size=(self.resize, self.resize), mode="bilinear", align_corners=False)
        outs0, outs1 = self.net(x0), self.net(x1)
        needs_grad = torch.is_grad_enabled() and (
            in0.requires_grad or in1.requires_grad or any(p.requires_grad for p in self.parameters()))
        dropout_active = self.training and any(isinstance(m, nn.Dropout) for m in self.modules())
        fused = not (self.spatial or needs_grad or dropout_active)
        res = []
        for k in range(len(self.chns)):
            if fused:
                res.append(ops.lpips_layer(outs0[k], outs1[k], self._lin_weight(k)).reshape(-1, 1, 1, 1))
                continue
            f0 = outs0[k] / (torch.sqrt((outs0[k] ** 2).sum(1, keepdim=True)) + 1e-8)
            f1 = outs1[k] / (torch.sqrt((outs1[k] ** 2).sum(1, keepdim=True)) + 1e-8)
            d = self.lins[k]((f0 - f1) ** 2)
            if self.spatial:
                res.append(nn.functional.interpolate(d, size=tuple(in0.shape[2:]), mode="bilinear", align_corners=False))
            else:
                res.append(d.mean(dim=(2, 3), keepdim=True))
        val = sum(res)
        return (val, res) if retperlayer else val


class _NoTrainLpips(_LPIPS):
    def train(self, mode: bool) -> "_NoTrainLpips":  # type: ignore[override]
        return super().train(False)


def _valid_img(img: Tensor, normalize: bool) -> bool:
    value_check = img.max() <= 1.0 and img.min() >= 0.0 if normalize else img.min() >= -1
    return img.ndim == 4 and img.shape[1] == 3 and bool(value_check)


def _lpips_update(img1: Tensor, img2: Tensor, net: nn.Module, normalize: bool) -> Tuple[Tensor, int]:
    if not (_valid_img(img1, normalize) and _valid_img(img2, normalize)):
        raise ValueError(
            "Expected both input arguments to be normalized tensors with shape [N, 3, H, W]."
            f" Got input with shape {img1.shape} and {img2.shape} and values in range"
            f" {[img1.min(), img1.max()]} and {[img2.min(), img2.max()]} when all values are"
            f" expected to be in the {[0, 1] if normalize else [-1, 1]} range.")
    return net(img1, img2, normalize=normalize).squeeze(), img1.shape[0]


def _lpips_compute(sum_scores: Tensor, total: Union[Tensor, int], reduction: str = "mean") -> Tensor:
    return sum_scores / total if reduction == "mean" else sum_scores


def learned_perceptual_image_patch_similarity(img1: Tensor, img2: Tensor,
                                              net_type: Literal["alex", "vgg", "squeeze"] = "alex",
                                              reduction: Literal["sum", "mean"] = "mean", normalize: bool = False,
                                              pretrained: bool = True, pnet_rand: bool = False,
                                              weights_path: Optional[str] = None,
                                              backbone_weights_path: Optional[str] = None) -> Tensor:
    """LPIPS between two image batches (``F/image/lpips.py:399``).  ``pretrained`` / ``pnet_rand`` /
    ``*weights_path`` control where weights come from (nothing is downloaded)."""
    net = _NoTrainLpips(pretrained=pretrained, net=net_type, pnet_rand=pnet_rand, model_path=weights_path,
                        backbone_weights_path=backbone_weights_path).to(device=img1.device, dtype=img1.dtype)
    loss, total = _lpips_update(img1, img2, net, normalize)
    return _lpips_compute(loss.sum(), total, reduction)
