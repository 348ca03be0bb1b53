"""MFMA NT-GEMM epilogues vs hipBLASLt (torch.matmul) and torch.cdist at the pairwise headline shapes.

One JSON line per (epilogue, shape): ``ours_ms``, ``tflops`` (2 N M D / t), and the vendor reference time.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd import ops  # noqa: E402


def timeit(fn, iters=10):
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
    for n, m, d in [(8192, 8192, 512), (4096, 4096, 2048), (16384, 16384, 256), (2048, 50000, 2048)]:
        x = torch.randn(n, d, device=dev, generator=g)
        y = torch.randn(m, d, device=dev, generator=g)
        nx, ny = (x * x).sum(1), (y * y).sum(1)
        ix, iy = 1 / x.norm(dim=1), 1 / y.norm(dim=1)
        flop = 2.0 * n * m * d
        st = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_STORE))
        eu = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_EUCLID, nx, ny))
        rm = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_ROW_MIN, ix, iy))
        mm = timeit(lambda: x @ y.T)
        cd = timeit(lambda: torch.cdist(x, y))
        # fused reduction epilogues vs the vendor GEMM followed by the same reduction in torch ops (the [N, M]
        # matrix written and read back): MiFID row-min of 1 - |cos|, KID polynomial-kernel sum, BERTScore row/col max
        xn, yn = x * ix[:, None], y * iy[:, None]
        rm_v = timeit(lambda: (1 - (xn @ yn.T).abs()).amin(1))
        ps = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_POLY_SUM, scale=1 / d, coef=1.0, degree=3).sum())
        ps_v = timeit(lambda: ((x @ y.T) / d + 1.0).pow(3).sum())
        rc = timeit(lambda: ops.gemm_row_col_max(x[None], y[None]))

        def rc_vendor():
            s_ = x @ y.T
            return s_.amax(1), s_.amax(0)

        rc_v = timeit(rc_vendor)
        print(json.dumps({"shape": [n, m, d], "store_ms": round(st, 4), "store_tflops": round(flop / st / 1e9, 1),
                          "euclid_fp32_ms": round(eu, 4), "hipblaslt_mm_ms": round(mm, 4),
                          "hipblaslt_tflops": round(flop / mm / 1e9, 1), "torch_cdist_ms": round(cd, 4),
                          "fused_rowmin_ms": round(rm, 4), "vendor_rowmin_ms": round(rm_v, 4),
                          "fused_polysum_ms": round(ps, 4), "vendor_polysum_ms": round(ps_v, 4),
                          "fused_rowcolmax_ms": round(rc, 4), "vendor_rowcolmax_ms": round(rc_v, 4),
                          "stages": os.environ.get("TM_AMD_GEMM_STAGES", "auto")}), flush=True)
        del x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
