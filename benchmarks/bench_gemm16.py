"""16-bit MFMA NT-GEMM (bf16 / fp16 operands, fp32 accumulate) vs hipBLASLt (torch.matmul in the same dtype) at the
pairwise / KID / BERTScore shapes.  One JSON line per (dtype, shape): our store (16-bit output) and fused epilogues
against the vendor GEMM (+ the same reduction in torch ops), and the full ``pairwise_cosine_similarity`` against the
reference's recipe (normalise in the input dtype, then a vendor GEMM: F/pairwise/cosine.py:24-46)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchmetrics_amd as tm  # noqa: E402
from torchmetrics_amd import ops  # noqa: E402


def timeit(fn, iters=20):
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
    shapes = [(8192, 8192, 512), (4096, 4096, 2048), (16384, 16384, 256), (2048, 50000, 2048), (2048, 2048, 768)]
    for dtype in (torch.bfloat16, torch.float16):
        for n, m, d in shapes:
            x = torch.randn(n, d, device=dev, generator=g).to(dtype)
            y = torch.randn(m, d, device=dev, generator=g).to(dtype)
            ix = 1 / torch.linalg.vector_norm(x, dim=1, dtype=torch.float32)
            iy = 1 / torch.linalg.vector_norm(y, dim=1, dtype=torch.float32)
            flop = 2.0 * n * m * d
            st = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_STORE, out_dtype=dtype))
            mm = timeit(lambda: x @ y.T)
            rc = timeit(lambda: ops.gemm_row_col_max(x[None], y[None]))

            def rc_vendor():
                s_ = x @ y.T
                return s_.amax(1), s_.amax(0)

            rc_v = timeit(rc_vendor)
            ps = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_POLY_SUM, scale=1 / d, coef=1.0, degree=3).sum())
            ps_v = timeit(lambda: ((x @ y.T).float() / d + 1.0).pow(3).sum())
            cos = timeit(lambda: tm.functional.pairwise_cosine_similarity(x, y))
            cos_gemm = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_COSINE, ix, iy, out_dtype=dtype))
            norms = timeit(lambda: ops.row_norms(x, inverse=True, y=y))

            def cos_ref():
                xn = x / torch.norm(x, p=2, dim=1).unsqueeze(1)
                yn = y / torch.norm(y, p=2, dim=1).unsqueeze(1)
                return xn @ yn.T

            cos_v = timeit(cos_ref)
            print(json.dumps({
                "dtype": str(dtype).split(".")[-1], "shape": [n, m, d],
                "store_ms": round(st, 4), "store_tflops": round(flop / st / 1e9, 1),
                "hipblaslt_ms": round(mm, 4), "hipblaslt_tflops": round(flop / mm / 1e9, 1),
                "fused_rowcolmax_ms": round(rc, 4), "vendor_rowcolmax_ms": round(rc_v, 4),
                "fused_polysum_ms": round(ps, 4), "vendor_polysum_ms": round(ps_v, 4),
                "pairwise_cosine_ms": round(cos, 4), "reference_recipe_cosine_ms": round(cos_v, 4),
                "cosine_gemm_only_ms": round(cos_gemm, 4), "row_norms_ms": round(norms, 4)}), flush=True)
            del x, y
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
