"""Pairwise similarity / distance matrices (reference ``F/pairwise/*.py``).

Distances (euclidean, manhattan, minkowski) run on the LDS-tiled HIP difference kernel
(:func:`torchmetrics_amd.ops.pairwise_distance`), which never materialises the reference's ``[N, M, d]`` broadcast
(``F/pairwise/manhattan.py:39``, ``minkowski.py:43``) and fuses root, ``zero_diagonal`` and the ``sum``/``mean`` row
reduction into the epilogue; euclidean (no reduction) is the reference's fp64 formula on the fp64 MFMA GEMM.
Similarities (linear, cosine) are plain GEMMs: small ones run on the MFMA kernel (``ops.gemm_nt``, fused scaling),
large ones on the vendor GEMM (hipBLASLt via ``torch.mm``, see ``_VENDOR_GEMM_MACS``); cosine row-normalises first
exactly like the reference (``F/pairwise/cosine.py:24-46``).
"""
from typing import Optional, Tuple

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.utilities.exceptions import TorchMetricsUserError

_Reduction = Optional[Literal["mean", "sum", "none"]]


def _check_input(x: Tensor, y: Optional[Tensor] = None,
                 zero_diagonal: Optional[bool] = None) -> Tuple[Tensor, Tensor, bool]:
    """Shape checks; ``y`` defaults to ``x`` (and ``zero_diagonal`` then defaults to True), ``F/pairwise/helpers.py``."""
    if x.ndim != 2:
        raise ValueError(f"Expected argument `x` to be a 2D tensor of shape `[N, d]` but got {x.shape}")
    if y is not None:
        if y.ndim != 2 or y.shape[1] != x.shape[1]:
            raise ValueError(
                "Expected argument `y` to be a 2D tensor of shape `[M, d]` where"
                " `d` should be same as the last dimension of `x`"
            )
        zero_diagonal = False if zero_diagonal is None else zero_diagonal
    else:
        y = x
        zero_diagonal = True if zero_diagonal is None else zero_diagonal
    return x, y, zero_diagonal


def _check_reduction(reduction: _Reduction) -> None:
    if reduction not in ("mean", "sum", "none", None):
        raise ValueError(f"Expected reduction to be one of `['mean', 'sum', None]` but got {reduction}")


def _reduce_distance_matrix(distmat: Tensor, reduction: _Reduction = None) -> Tensor:
    _check_reduction(reduction)
    if reduction == "mean":
        return distmat.mean(dim=-1)
    if reduction == "sum":
        return distmat.sum(dim=-1)
    return distmat


def _safe_matmul(x: Tensor, y: Tensor) -> Tensor:
    """``x @ y.T``; half precision on CPU is upcast (no CPU half GEMM)."""
    if x.dtype in (torch.float16, torch.bfloat16) and x.device.type == "cpu":
        return (x.float() @ y.T.float()).to(x.dtype)
    return x @ y.T


def _zero_diag(d: Tensor, zero_diagonal: bool) -> Tensor:
    if zero_diagonal:
        d.fill_diagonal_(0)
    return d


def _mfma_ok(x: Tensor) -> bool:
    """ROCm, non-fp64 operands with 16-byte rows: the matrix-core GEMM path (``ops.gemm_nt``: fp32 MFMA, or the 16-bit
    MFMA for bf16 / fp16 operands)."""
    return x.is_cuda and x.dtype != torch.float64 and x.shape[-1] % 4 == 0 and x.shape[-1] > 0


# plain (store-epilogue) GEMMs of at least this many multiply-adds go to the vendor GEMM (hipBLASLt via torch.mm):
# past the launch-overhead regime its tuned kernels are faster than ours for a plain store (bench_pairwise.py: 8192^2 x
# 512 0.52 vs 0.62 ms, 4096^2 x 128 0.048 vs 0.060 ms); below it our MFMA kernel wins (512^2 x 64: 0.011 vs 0.021 ms).
# Fused REDUCTION epilogues (KID / MiFID / BERTScore / row sums) stay on ops.gemm_nt: no [N, M] round trip.
_VENDOR_GEMM_MACS = 1 << 30


def _vendor_gemm(x: Tensor, y: Tensor) -> bool:
    """fp32 store GEMMs past the launch-overhead regime.  bf16 / fp16 operands always run our 16-bit MFMA kernel."""
    return (x.is_cuda and x.dtype == torch.float32 and y.dtype == torch.float32
            and x.shape[0] * y.shape[0] * x.shape[1] >= _VENDOR_GEMM_MACS)


def _euclid_ok(x: Tensor) -> bool:
    """ROCm, non-empty rows, non-fp64 inputs: the fp64 matrix-core GEMM path (``ops.euclid_f64``, fp32 output).  fp64
    inputs keep the fp64 difference kernel (``ops.pairwise_distance``), which returns fp64 distances."""
    return x.is_cuda and x.dtype != torch.float64 and x.shape[-1] > 0


def _euclid_mfma(x: Tensor, y: Tensor, zd: bool) -> Tensor:
    """The reference's fp64 formula (``F/pairwise/euclidean.py:35-44``) in one fp64-MFMA launch with an fp32 epilogue:
    near-duplicate rows keep the fp64 cancellation accuracy (an fp32 GEMM would lose ~1e-7 * |x|^2 of it)."""
    d = ops.euclid_f64(x, y, zd)
    return d if x.dtype == torch.float32 else d.to(x.dtype)


def _distance(x: Tensor, y: Optional[Tensor], metric: int, p: float, reduction: _Reduction,
              zero_diagonal: Optional[bool]) -> Tensor:
    _check_reduction(reduction)
    x, y, zd = _check_input(x, y, zero_diagonal)
    red = reduction if reduction in ("sum", "mean") else None
    if metric == ops.PW_L2 and red is None and _euclid_ok(x):
        return _euclid_mfma(x, y, zd)
    return ops.pairwise_distance(x, y, metric, p, zd, red)


def _pairwise_euclidean_distance_update(x: Tensor, y: Optional[Tensor] = None,
                                        zero_diagonal: Optional[bool] = None) -> Tensor:
    x, y, zd = _check_input(x, y, zero_diagonal)
    if _euclid_ok(x):
        return _euclid_mfma(x, y, zd)
    return ops.pairwise_distance(x, y, ops.PW_L2, 2.0, zd, None)


def pairwise_euclidean_distance(x: Tensor, y: Optional[Tensor] = None, reduction: _Reduction = None,
                                zero_diagonal: Optional[bool] = None) -> Tensor:
    """``||x_i - y_j||_2`` for every pair of rows (``F/pairwise/euclidean.py:47``)."""
    return _distance(x, y, ops.PW_L2, 2.0, reduction, zero_diagonal)


def _pairwise_manhattan_distance_update(x: Tensor, y: Optional[Tensor] = None,
                                        zero_diagonal: Optional[bool] = None) -> Tensor:
    x, y, zd = _check_input(x, y, zero_diagonal)
    return ops.pairwise_distance(x, y, ops.PW_L1, 1.0, zd, None)


def pairwise_manhattan_distance(x: Tensor, y: Optional[Tensor] = None, reduction: _Reduction = None,
                                zero_diagonal: Optional[bool] = None) -> Tensor:
    """``||x_i - y_j||_1`` for every pair of rows (``F/pairwise/manhattan.py:41``)."""
    return _distance(x, y, ops.PW_L1, 1.0, reduction, zero_diagonal)


def _pairwise_minkowski_distance_update(x: Tensor, y: Optional[Tensor] = None, exponent: float = 2,
                                        zero_diagonal: Optional[bool] = None) -> Tensor:
    x, y, zd = _check_input(x, y, zero_diagonal)
    if not (isinstance(exponent, (float, int)) and exponent >= 1):
        raise TorchMetricsUserError(f"Argument ``p`` must be a float or int greater than 1, but got {exponent}")
    metric = ops.PW_L1 if exponent == 1 else (ops.PW_L2 if exponent == 2 else ops.PW_LP)
    return ops.pairwise_distance(x, y, metric, float(exponent), zd, None)


def pairwise_minkowski_distance(x: Tensor, y: Optional[Tensor] = None, exponent: float = 2,
                                reduction: _Reduction = None, zero_diagonal: Optional[bool] = None) -> Tensor:
    """``||x_i - y_j||_p`` for every pair of rows (``F/pairwise/minkowski.py:49``)."""
    if not (isinstance(exponent, (float, int)) and exponent >= 1):
        raise TorchMetricsUserError(f"Argument ``p`` must be a float or int greater than 1, but got {exponent}")
    metric = ops.PW_L1 if exponent == 1 else (ops.PW_L2 if exponent == 2 else ops.PW_LP)
    return _distance(x, y, metric, float(exponent), reduction, zero_diagonal)


def _pairwise_linear_similarity_update(x: Tensor, y: Optional[Tensor] = None,
                                       zero_diagonal: Optional[bool] = None) -> Tensor:
    x, y, zd = _check_input(x, y, zero_diagonal)
    if _mfma_ok(x) and not _vendor_gemm(x, y):
        return ops.gemm_nt(x, y, ops.GEMM_STORE, zero_diagonal=zd, out_dtype=x.dtype)
    return _zero_diag(_safe_matmul(x, y), zd)


def pairwise_linear_similarity(x: Tensor, y: Optional[Tensor] = None, reduction: _Reduction = None,
                               zero_diagonal: Optional[bool] = None) -> Tensor:
    """``<x_i, y_j>`` for every pair of rows (``F/pairwise/linear.py:42``)."""
    _check_reduction(reduction)
    return _reduce_distance_matrix(_pairwise_linear_similarity_update(x, y, zero_diagonal), reduction)


def _pairwise_cosine_similarity_update(x: Tensor, y: Optional[Tensor] = None,
                                       zero_diagonal: Optional[bool] = None) -> Tensor:
    x, y, zd = _check_input(x, y, zero_diagonal)
    if _mfma_ok(x) and not _vendor_gemm(x, y):
        # fp32 inverse norms read straight from the operand (one wave per row, no upcast copy)
        if y is x:
            ix = iy = ops.row_norms(x, inverse=True)
        else:
            ix, iy = ops.row_norms(x, inverse=True, y=y)
        return ops.gemm_nt(x, y, ops.GEMM_COSINE, ix, iy, zero_diagonal=zd, out_dtype=x.dtype)
    xn = x / torch.linalg.vector_norm(x, 2, dim=1, keepdim=True)
    yn = xn if y is x else y / torch.linalg.vector_norm(y, 2, dim=1, keepdim=True)
    return _zero_diag(_safe_matmul(xn, yn), zd)


def pairwise_cosine_similarity(x: Tensor, y: Optional[Tensor] = None, reduction: _Reduction = None,
                               zero_diagonal: Optional[bool] = None) -> Tensor:
    """``<x_i, y_j> / (||x_i|| ||y_j||)`` for every pair of rows (``F/pairwise/cosine.py:48``)."""
    _check_reduction(reduction)
    return _reduce_distance_matrix(_pairwise_cosine_similarity_update(x, y, zero_diagonal), reduction)


__all__ = [
    "pairwise_cosine_similarity",
    "pairwise_euclidean_distance",
    "pairwise_linear_similarity",
    "pairwise_manhattan_distance",
    "pairwise_minkowski_distance",
]
