"""Pairwise distance kernels vs the reference's formulations on the same device.

For each metric times our call (HIP difference kernel for euclidean / manhattan / minkowski, vendor GEMM for linear /
cosine) against the reference's arithmetic re-expressed with plain torch ops (fp64 norm-expansion GEMM for euclidean,
``[N, M, d]`` broadcast for manhattan / minkowski, ``F/pairwise/*.py``) and ``torch.cdist``.  Prints one JSON line per
(metric, shape).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd import functional as F  # noqa: E402
from torchmetrics_amd import ops  # noqa: E402


def ref_euclid(x, y):
    xd, yd = x.double(), y.double()
    d = ((xd * xd).sum(1, keepdim=True) + (yd * yd).sum(1) - 2 * xd.mm(yd.T)).to(x.dtype)
    return d.sqrt()


def ref_manhattan(x, y):
    return (x.unsqueeze(1) - y.unsqueeze(0).repeat(x.shape[0], 1, 1)).abs().sum(dim=-1)


def ref_minkowski(x, y, p=3.0):
    xd, yd = x.double(), y.double()
    return (xd.unsqueeze(1) - yd.unsqueeze(0)).abs().pow(p).sum(-1).pow(1.0 / p).to(x.dtype)


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [(4096, 4096, 128), (8192, 8192, 512), (512, 512, 64)]
    for n, m, d in shapes:
        x = torch.randn(n, d, device=dev, generator=g)
        y = torch.randn(m, d, device=dev, generator=g)
        iters = 5 if n >= 8192 else 20
        nx, ny = (x * x).sum(1), (y * y).sum(1)
        cases = [
            ("euclidean_fp32_mfma_r2", lambda: ops.gemm_nt(x, y, ops.GEMM_EUCLID, nx, ny), None, None),
            ("euclidean", lambda: F.pairwise_euclidean_distance(x, y), lambda: ref_euclid(x, y),
             lambda: torch.cdist(x, y)),
            ("manhattan", lambda: F.pairwise_manhattan_distance(x, y),
             (lambda: ref_manhattan(x, y)) if n * m * d * 4 < 8e9 else None, lambda: torch.cdist(x, y, p=1)),
            ("minkowski3", lambda: F.pairwise_minkowski_distance(x, y, exponent=3),
             (lambda: ref_minkowski(x, y)) if n * m * d * 8 < 8e9 else None, lambda: torch.cdist(x, y, p=3)),
            ("euclidean_mean", lambda: F.pairwise_euclidean_distance(x, y, reduction="mean"),
             lambda: ref_euclid(x, y).mean(-1), None),
            ("linear", lambda: F.pairwise_linear_similarity(x, y), lambda: x @ y.T, None),
            ("cosine", lambda: F.pairwise_cosine_similarity(x, y), None, None),
        ]
        for name, ours, ref, cd in cases:
            rec = {"bench": "pairwise", "metric": name, "shape": [n, m, d], "ours_ms": round(timeit(ours, iters), 4)}
            if ref is not None:
                rec["reference_formula_ms"] = round(timeit(ref, iters), 4)
                rec["speedup_vs_reference"] = round(rec["reference_formula_ms"] / rec["ours_ms"], 2)
            if cd is not None:
                try:
                    rec["torch_cdist_ms"] = round(timeit(cd, iters), 4)
                except RuntimeError as err:  # torch.cdist p != 2 launch fails for large shapes on ROCm
                    rec["torch_cdist_error"] = str(err).splitlines()[0]
            if name in ("euclidean", "manhattan", "minkowski3"):
                rec["ours_gelem_per_s"] = round(n * m * d / rec["ours_ms"] / 1e6, 1)
            print(json.dumps(rec), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
