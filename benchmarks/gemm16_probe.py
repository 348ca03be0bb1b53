"""Timing of the 16-bit GEMM store path at two shapes (kept for the round-6 loop probes: profiles/r06_gemm16_loop_probes.txt)."""
import sys, os, time, json, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from torchmetrics_amd import ops
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
for n, m, d in [(4096, 4096, 2048), (16384, 16384, 256)]:
    x = torch.randn(n, d, device=dev, generator=g).to(torch.bfloat16)
    y = torch.randn(m, d, device=dev, generator=g).to(torch.bfloat16)
    f = lambda: ops.gemm_nt(x, y, ops.GEMM_STORE, out_dtype=torch.bfloat16)
    for _ in range(3): f()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(20): f()
    torch.cuda.synchronize(); ms = (time.perf_counter() - t) / 20 * 1e3
    print(json.dumps({"pp": os.environ.get("TM_AMD_GEMM16_PP"), "shape": [n, m, d], "ms": round(ms, 4), "tf": round(2*n*m*d/ms/1e9, 1)}), flush=True)
