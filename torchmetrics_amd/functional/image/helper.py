"""Window / padding helpers for the image metrics (behaviour of reference ``F/image/helper.py``)."""
from typing import Sequence, Tuple, Union

import torch
import torch.nn.functional as F  # noqa: N812
from torch import Tensor


def _gaussian(kernel_size: int, sigma: float, dtype: torch.dtype, device: Union[torch.device, str]) -> Tensor:
    """Normalised 1-D Gaussian taps, shape ``(1, kernel_size)``."""
    half = (kernel_size - 1) / 2
    dist = torch.linspace(-half, half, kernel_size, dtype=dtype, device=device)
    g = torch.exp(-0.5 * (dist / sigma) ** 2)
    return (g / g.sum()).unsqueeze(0)


def _gaussian_kernel_2d(channel: int, kernel_size: Sequence[int], sigma: Sequence[float], dtype: torch.dtype,
                        device: Union[torch.device, str]) -> Tensor:
    gx = _gaussian(kernel_size[0], sigma[0], dtype, device)
    gy = _gaussian(kernel_size[1], sigma[1], dtype, device)
    return (gx.t() @ gy).expand(channel, 1, kernel_size[0], kernel_size[1])


def _gaussian_kernel_3d(channel: int, kernel_size: Sequence[int], sigma: Sequence[float], dtype: torch.dtype,
                        device: Union[torch.device, str]) -> Tensor:
    gx, gy, gz = (_gaussian(k, s, dtype, device)[0] for k, s in zip(kernel_size, sigma))
    k = gx[:, None, None] * gy[None, :, None] * gz[None, None, :]
    return k.expand(channel, 1, *kernel_size)


def _symmetric_pad(inputs: Tensor, dim: int, before: int, after: int) -> Tensor:
    """Edge-inclusive mirror padding ("symmetric") of ``before`` / ``after`` elements along ``dim``."""
    n = inputs.shape[dim]
    parts = []
    if before > 0:
        parts.append(inputs.narrow(dim, 0, before).flip(dim))
    parts.append(inputs)
    if after > 0:
        parts.append(inputs.narrow(dim, n - after, after).flip(dim))
    return torch.cat(parts, dim)


def _reflection_pad_2d(inputs: Tensor, pad: int, outer_pad: int = 0) -> Tensor:
    """Reference's uniform-filter padding: ``pad`` mirrored elements before, ``pad + outer_pad - 1`` after."""
    for dim in (2, 3):
        inputs = _symmetric_pad(inputs, dim, pad, pad + outer_pad - 1)
    return inputs


def _reflection_pad_3d(inputs: Tensor, pad_h: int, pad_w: int, pad_d: int) -> Tensor:
    return F.pad(inputs, (pad_h, pad_h, pad_w, pad_w, pad_d, pad_d), mode="reflect")


def _uniform_filter(inputs: Tensor, window_size: int) -> Tensor:
    """Per-channel box filter (one grouped convolution over all channels), output size == input size."""
    padded = _reflection_pad_2d(inputs, window_size // 2, window_size % 2)
    c = inputs.shape[1]
    w = torch.full((c, 1, window_size, window_size), 1.0 / window_size**2, dtype=inputs.dtype, device=inputs.device)
    return F.conv2d(padded, w, groups=c)


def _window_1d(kernel_size: Sequence[int], sigma: Sequence[float], gaussian: bool, dtype: torch.dtype,
               device: torch.device) -> Tuple[Tensor, Tensor]:
    """Separable window taps (rows, cols) for the fused SSIM / UQI kernel."""
    if gaussian:
        return _gaussian(kernel_size[0], sigma[0], dtype, device)[0], _gaussian(kernel_size[1], sigma[1], dtype,
                                                                                 device)[0]
    return (torch.full((kernel_size[0],), 1.0 / kernel_size[0], dtype=dtype, device=device),
            torch.full((kernel_size[1],), 1.0 / kernel_size[1], dtype=dtype, device=device))
