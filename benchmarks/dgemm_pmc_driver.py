"""Driver for PMC passes over the fp64 matrix-core GEMM (ops.dgemm: one problem and the Newton-Schulz batched pair) vs
torch.matmul (Tensile) at one FID shape (run under rocprofv3 --pmc).  Usage: dgemm_pmc_driver.py [d]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd import ops  # noqa: E402


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(d, d, dtype=torch.float64, device="cuda", generator=g)
    b = torch.randn(d, d, dtype=torch.float64, device="cuda", generator=g)
    c, c2 = torch.empty_like(a), torch.empty_like(a)
    for _ in range(3):
        ops.dgemm(a, b, c)
    for _ in range(3):
        ops.dgemm([a, b], [b, a], [c, c2], alpha=[1.0, 1.0], beta=[0.5, 0.5], cin=[a, b])
    for _ in range(3):
        torch.matmul(a, b, out=c2)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
