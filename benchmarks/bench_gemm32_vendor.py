"""fp32 store GEMM (ops.gemm_nt) vs hipBLASLt at the four pairwise shapes (the measurement behind _VENDOR_GEMM_MACS)."""
import sys, os, time, json, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from torchmetrics_amd import ops
g = torch.Generator(device="cuda").manual_seed(0)
for n, m, d in [(4096, 4096, 2048), (8192, 8192, 512), (16384, 16384, 256), (2048, 50000, 2048)]:
    x = torch.randn(n, d, device="cuda", generator=g); y = torch.randn(m, d, device="cuda", generator=g)
    def t(f):
        for _ in range(3): f()
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(10): f()
        torch.cuda.synchronize(); return (time.perf_counter() - t0) / 10 * 1e3
    a = t(lambda: ops.gemm_nt(x, y, ops.GEMM_STORE)); b = t(lambda: x @ y.T)
    print(json.dumps({"probe": os.environ.get("TM_AMD_GEMM_PROBE16"), "shape": [n, m, d], "ours_ms": round(a, 4), "hipblaslt_ms": round(b, 4)}), flush=True)
