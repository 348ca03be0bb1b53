"""Driver for PMC passes over the bf16 NT-GEMM (ours: ops.gemm_nt store, 16-bit output) vs hipBLASLt at one shape
(run under rocprofv3 --pmc).  Usage: gemm16_pmc_driver.py [n m d]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd import ops  # noqa: E402


def main():
    n, m, d = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (4096, 4096, 2048)))
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(n, d, device="cuda", generator=g).to(torch.bfloat16)
    y = torch.randn(m, d, device="cuda", generator=g).to(torch.bfloat16)
    for _ in range(3):
        ops.gemm_nt(x, y, ops.GEMM_STORE, out_dtype=torch.bfloat16)
        x @ y.T
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
