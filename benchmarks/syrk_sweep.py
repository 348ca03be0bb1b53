"""Sweep the fp64 SYRK (FID feature statistics) over batch size and split-K count; prints JSON lines with achieved
fp64 TFLOP/s on the useful (upper-triangle) FLOPs and the reference formulation (``x.double().t().mm(...)``)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchmetrics_amd import ops  # noqa: E402

D = int(os.environ.get("SWEEP_D", "2048"))


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    s = torch.zeros(D, dtype=torch.float64, device="cuda")
    c = torch.zeros(D, D, dtype=torch.float64, device="cuda")
    for b in (1000, 4096, 16384, 50000):
        x = torch.randn(b, D, device="cuda")
        reps = max(3, 200000 // b)
        useful = b * D * (D + 1)  # upper triangle incl. diagonal, 2 FLOP per MAC
        ref = timeit(lambda: c.add_(x.double().t().mm(x.double())), reps)
        print(json.dumps({"b": b, "impl": "reference_dgemm", "us": round(ref * 1e6, 1),
                          "tflops_useful": round(useful / ref / 1e12, 1)}), flush=True)
        for sp in ("auto", "1", "2", "4", "7", "8", "15", "16", "32"):
            if sp == "auto":
                os.environ.pop("TM_AMD_SYRK_SPLITS", None)
            else:
                os.environ["TM_AMD_SYRK_SPLITS"] = sp
            t = timeit(lambda: ops.feature_moments_update(x, s, c), reps)
            print(json.dumps({"b": b, "splits": sp, "us": round(t * 1e6, 1),
                              "tflops_useful": round(useful / t / 1e12, 1)}), flush=True)
        os.environ.pop("TM_AMD_SYRK_SPLITS", None)


if __name__ == "__main__":
    main()
