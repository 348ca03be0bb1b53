"""One 16-bit NT-GEMM shape for counter / trace runs: ours (store, 16-bit output) and hipBLASLt (x @ y.T), 5 calls
each.  ``--shape N M D``, ``--dtype bf16|fp16``, ``--kind store|cosine``."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=3, default=[8192, 8192, 512])
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--kind", default="store")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    n, m, d = a.shape
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(n, d, device="cuda", generator=g).to(dt)
    y = torch.randn(m, d, device="cuda", generator=g).to(dt)
    kind = ops.GEMM_STORE
    for _ in range(a.iters):
        ops.gemm_nt(x, y, kind, out_dtype=dt)
        x @ y.T
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
