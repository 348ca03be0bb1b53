"""Store-epilogue MFMA NT-GEMM time at the pairwise headline shapes (for TM_AMD_GEMM_BK / TM_AMD_GEMM_STAGES sweeps)
next to hipBLASLt (torch.matmul).  One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_gemm import timeit  # noqa: E402
from torchmetrics_amd import ops  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    for n, m, d in [(8192, 8192, 512), (4096, 4096, 2048), (16384, 16384, 256), (2048, 50000, 2048)]:
        x = torch.randn(n, d, device="cuda", generator=g)
        y = torch.randn(m, d, device="cuda", generator=g)
        ref = (x[:64] @ y[:64].T)
        out = ops.gemm_nt(x[:64].contiguous(), y[:64].contiguous(), ops.GEMM_STORE)
        err = float((out - ref).abs().max())
        st = timeit(lambda: ops.gemm_nt(x, y, ops.GEMM_STORE))
        mm = timeit(lambda: x @ y.T)
        f = 2.0 * n * m * d
        print(json.dumps({"shape": [n, m, d], "bk": os.environ.get("TM_AMD_GEMM_BK", "auto"),
                          "stages": os.environ.get("TM_AMD_GEMM_STAGES", "auto"), "ours_tflops": round(f / st / 1e9, 1),
                          "hipblaslt_tflops": round(f / mm / 1e9, 1), "max_abs_err_64x64": err}), flush=True)
        del x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
