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
        flop = 2.0 * n * m * d
        st = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_STORE))
        eu = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_EUCLID, nx, ny))
        rm = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_ROW_MIN, nx, ny))
        mm = timeit(lambda: x @ y.T)
        cd = timeit(lambda: torch.cdist(x, y))
        print(json.dumps({"shape": [n, m, d], "store_ms": round(st, 4), "store_tflops": round(flop / st / 1e9, 1),
                          "euclid_ms": round(eu, 4), "rowmin_ms": round(rm, 4),
                          "rowmin_tflops": round(flop / rm / 1e9, 1), "hipblaslt_mm_ms": round(mm, 4),
                          "hipblaslt_tflops": round(flop / mm / 1e9, 1), "torch_cdist_ms": round(cd, 4),
                          "stages": os.environ.get("TM_AMD_GEMM_STAGES", "2")}), flush=True)


if __name__ == "__main__":
    main()
