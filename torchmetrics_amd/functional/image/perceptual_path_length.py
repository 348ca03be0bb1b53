"""Perceptual path length (reference ``F/image/perceptual_path_length.py``): LPIPS distance between generator
outputs at latents ``z`` and ``I(z, z', eps)``, scaled by ``1/eps^2``, outlier-trimmed by quantiles.  Both halves of
a batch go through the generator in one call; the LPIPS distance uses the fused layer kernel."""
import math
from typing import Literal, Optional, Tuple, Union

import torch
from torch import Tensor, nn

from torchmetrics_amd.functional.image.lpips import _LPIPS


class GeneratorType(nn.Module):
    """Interface: ``sample(num_samples) -> [num_samples, z_size]`` and (conditional) ``num_classes``."""

    @property
    def num_classes(self) -> int:
        raise NotImplementedError

    def sample(self, num_samples: int) -> Tensor:
        raise NotImplementedError


def _validate_generator_model(generator: GeneratorType, conditional: bool = False) -> None:
    if not hasattr(generator, "sample"):
        raise NotImplementedError(
            "The generator must have a `sample` method with signature `sample(num_samples: int) -> Tensor` where the"
            " returned tensor has shape `(num_samples, z_size)`.")
    if not callable(generator.sample):
        raise ValueError("The generator's `sample` method must be callable.")
    if conditional and not hasattr(generator, "num_classes"):
        raise AttributeError("The generator must have a `num_classes` attribute when `conditional=True`.")
    if conditional and not isinstance(generator.num_classes, int):
        raise ValueError("The generator's `num_classes` attribute must be an integer when `conditional=True`.")


_INTERPOLATIONS = ("lerp", "slerp_any", "slerp_unit")
_SIM_NETS = ("alex", "vgg", "squeeze")


def _perceptual_path_length_validate_arguments(num_samples: int = 10_000, conditional: bool = False,
                                               batch_size: int = 128, interpolation_method: str = "lerp",
                                               epsilon: float = 1e-4, resize: Optional[int] = 64,
                                               lower_discard: Optional[float] = 0.01,
                                               upper_discard: Optional[float] = 0.99) -> None:
    """Argument checks with the reference's messages (``F/image/perceptual_path_length.py:65-104``), table-driven."""
    rules = [
        (isinstance(num_samples, int) and num_samples > 0,
         f"Argument `num_samples` must be a positive integer, but got {num_samples}."),
        (isinstance(conditional, bool), f"Argument `conditional` must be a boolean, but got {conditional}."),
        (isinstance(batch_size, int) and batch_size > 0,
         f"Argument `batch_size` must be a positive integer, but got {batch_size}."),
        (interpolation_method in _INTERPOLATIONS,
         f"Argument `interpolation_method` must be one of 'lerp', 'slerp_any', 'slerp_unit',got {interpolation_method}."),
        (isinstance(epsilon, float) and epsilon > 0, f"Argument `epsilon` must be a positive float, but got {epsilon}."),
        (resize is None or (isinstance(resize, int) and resize > 0),
         f"Argument `resize` must be a positive integer or `None`, but got {resize}."),
    ]
    for name, v in (("lower_discard", lower_discard), ("upper_discard", upper_discard)):
        rules.append((v is None or (isinstance(v, float) and 0 <= v <= 1),
                      f"Argument `{name}` must be a float between 0 and 1 or `None`, but got {v}."))
    for ok, msg in rules:
        if not ok:
            raise ValueError(msg)


def _unit(x: Tensor, eps: float) -> Tensor:
    return x / (x * x).sum(dim=-1, keepdim=True).sqrt().clamp_min(eps)


def _interpolate(latents1: Tensor, latents2: Tensor, epsilon: float = 1e-4,
                 interpolation_method: Literal["lerp", "slerp_any", "slerp_unit"] = "lerp") -> Tensor:
    """Point at fraction ``epsilon`` from ``latents1`` towards ``latents2``.

    ``lerp``: straight line.  ``slerp_any``: along the great circle through the two directions, with the endpoints'
    own norms as weights (falls back to ``lerp`` for (anti)parallel or zero latents).  ``slerp_unit``: the slerp point
    projected back onto the unit sphere."""
    if latents1.shape != latents2.shape:
        raise ValueError("Latents must have the same shape.")
    if interpolation_method not in _INTERPOLATIONS:
        raise ValueError(
            f"Interpolation method {interpolation_method} not supported. Choose from 'lerp', 'slerp_any', 'slerp_unit'.")
    line = torch.lerp(latents1, latents2, epsilon)
    if interpolation_method == "lerp":
        return line
    tiny = 1e-7
    u1, u2 = _unit(latents1, tiny), _unit(latents2, tiny)
    cos = (u1 * u2).sum(dim=-1, keepdim=True)
    omega = cos.acos()
    inv_sin = 1.0 / omega.sin().clamp_min(tiny)
    arc = torch.sin((1 - epsilon) * omega) * inv_sin * latents1 + torch.sin(epsilon * omega) * inv_sin * latents2
    # a zero latent or (anti)parallel directions make the arc undefined: those rows take the straight line
    degenerate = (u1.norm(dim=-1, keepdim=True) < tiny) | (u2.norm(dim=-1, keepdim=True) < tiny) | \
        (cos.abs() > 1 - tiny)
    out = torch.where(degenerate, line, arc)
    return _unit(out, tiny) if interpolation_method == "slerp_unit" else out


def _resolve_sim_net(sim_net: Union[nn.Module, str], resize: Optional[int], device: torch.device) -> nn.Module:
    if isinstance(sim_net, nn.Module):
        return sim_net.to(device)
    if sim_net in _SIM_NETS:
        return _LPIPS(pretrained=True, net=sim_net, resize=resize).to(device)
    raise ValueError(f"sim_net must be a nn.Module or one of 'alex', 'vgg', 'squeeze', got {sim_net}")


def _quantile_trim(d: Tensor, lower_discard: Optional[float], upper_discard: Optional[float]) -> Tensor:
    """Keep the values between the two "lower"-interpolated quantiles, on the device: one sort gives both order
    statistics (``torch.quantile(..., interpolation="lower")`` is the element at ``floor(q (n - 1))``).  Without a
    lower quantile the floor is 0 (negative distances dropped) and without an upper one nothing is cut above, as in
    the reference."""
    n = d.numel()
    srt = d.sort().values
    lo = srt[int(math.floor(lower_discard * (n - 1)))] if lower_discard is not None else 0.0
    keep = d >= lo
    if upper_discard is not None:
        keep &= d <= srt[int(math.floor(upper_discard * (n - 1)))]
    return d[keep]


def perceptual_path_length(generator: GeneratorType, num_samples: int = 10_000, conditional: bool = False,
                           batch_size: int = 64, interpolation_method: Literal["lerp", "slerp_any", "slerp_unit"] = "lerp",
                           epsilon: float = 1e-4, resize: Optional[int] = 64, lower_discard: Optional[float] = 0.01,
                           upper_discard: Optional[float] = 0.99,
                           sim_net: Union[nn.Module, Literal["alex", "vgg", "squeeze"]] = "vgg",
                           device: Union[str, torch.device] = "cpu") -> Tuple[Tensor, Tensor, Tensor]:
    """(mean, std, kept distances) of the perceptual path length (API of ``F/image/perceptual_path_length.py:150``).

    Every latent pair ``(z, I(z, z', eps))`` is drawn up front; each batch sends both halves through the generator
    as ONE call and writes its LPIPS distances (scaled by ``1 / eps²``) into a preallocated device buffer, and the
    quantile trim runs on the device -- no per-batch host work beyond the generator / network calls."""
    _perceptual_path_length_validate_arguments(num_samples, conditional, batch_size, interpolation_method, epsilon,
                                               resize, lower_discard, upper_discard)
    _validate_generator_model(generator, conditional)
    device = torch.device(device)
    generator = generator.to(device)
    start = generator.sample(num_samples).to(device)
    end = _interpolate(start, generator.sample(num_samples).to(device), epsilon, interpolation_method)
    labels = torch.randint(0, generator.num_classes, (num_samples,)).to(device) if conditional else None
    net = _resolve_sim_net(sim_net, resize, device)
    scale = 1.0 / (epsilon * epsilon)
    with torch.inference_mode():
        dist = torch.empty(num_samples, device=device)
        for lo in range(0, num_samples, batch_size):
            hi = min(lo + batch_size, num_samples)
            pair = torch.cat((start[lo:hi], end[lo:hi]))
            imgs = generator(pair, labels[lo:hi].repeat(2)) if conditional else generator(pair)
            # generator outputs are in [0, 255]; LPIPS takes [-1, 1]
            imgs = imgs * (2.0 / 255.0) - 1.0
            a, b = imgs[: hi - lo], imgs[hi - lo:]
            dist[lo:hi] = net(a, b).reshape(-1).to(dist.dtype) * scale
        kept = _quantile_trim(dist, lower_discard, upper_discard)
        return kept.mean(), kept.std(), kept
