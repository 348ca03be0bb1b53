"""fp64 GEMM throughput: our matrix-core kernel (``ops.dgemm``) vs torch.matmul (rocBLAS / Tensile) at FID shapes.
Prints one JSON line per (shape, impl)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd import ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda")
    for d in (2048, 1024, 4096):
        a = torch.randn(d, d, dtype=torch.float64, device=dev)
        b = torch.randn(d, d, dtype=torch.float64, device=dev)
        c = torch.empty_like(a)
        c2 = torch.empty_like(a)
        flops = 2.0 * d ** 3
        ms_ours = timed(lambda: ops.dgemm(a, b, c))
        ref = a @ b
        err = float(((c - ref).abs().max() / ref.abs().max()).item())
        ms_batch = timed(lambda: ops.dgemm([a, b], [b, a], [c, c2], alpha=[1.0, 1.0], beta=[0.5, 0.5], cin=[a, b]))
        ms_ref = timed(lambda: torch.matmul(a, b, out=c2))
        for impl, ms, f in (("ours", ms_ours, flops), ("ours_batched2", ms_batch, 2 * flops), ("torch_matmul", ms_ref, flops)):
            print(json.dumps({"d": d, "impl": impl, "variant": os.environ.get("TM_AMD_DGEMM_VARIANT", "auto"), "ms": round(ms, 4), "tflops": round(f / ms / 1e9, 2),
                              "rel_err_vs_torch": err if impl == "ours" else None}), flush=True)


if __name__ == "__main__":
    main()
