"""One 4096 x 4096 x 2048 fp32 NT GEMM, ours (csrc/pairwise/gemm_nt.hip, 256 x 256 kernel) and hipBLASLt (torch.mm),
10 calls each -- for counter collection."""
import torch

from torchmetrics_amd import ops

g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(4096, 2048, device="cuda", generator=g)
y = torch.randn(4096, 2048, device="cuda", generator=g)
for _ in range(10):
    ops.gemm_nt(x, y, ops.GEMM_STORE)
    torch.mm(x, y.T)
torch.cuda.synchronize()
