"""FID compute breakdown on the 50k x 2048 bench covariances: power-iteration floor estimates, schedule length and
time of each part of the Newton-Schulz trace-sqrt.  One JSON line."""
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd.image import generative as G  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    n, d = 50_000, 2048
    f1 = torch.randn(n, d, device="cuda", generator=g).double()
    f2 = (torch.randn(n, d, device="cuda", generator=g) * 1.1 + 0.05).double()
    s1, s2 = torch.cov(f1.T), torch.cov(f2.T)
    del f1, f2
    p = s1 @ s2
    c = torch.minimum(torch.minimum(p.diagonal().sum(), p.abs().sum(1).max()), p.abs().sum(0).max())
    a0 = p / c
    v0 = torch.rand(d, 4, dtype=p.dtype, device=p.device, generator=torch.Generator(device="cuda").manual_seed(0))
    out = {}
    for iters in (6, 12, 24):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p1, p2 = G._ns_floor(a0, v0, iters=iters).tolist()
        out[f"floor_{iters}"] = {"p_first": p1, "p_second": p2, "ms": 1e3 * (time.perf_counter() - t0)}
    ev = torch.linalg.eigvals(p).real
    out["p_min_true"] = float(ev.min() / c)
    for low in (0.5 * math.sqrt(max(out["floor_24"]["p_second"], 0)), 1e-6):
        out[f"schedule_len_{low:.3g}"] = len(G._ns_schedule(low))
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        v = G._trace_sqrt_newton_schulz(s1, s2)
        torch.cuda.synchronize()
        out["ns_ms"] = 1e3 * (time.perf_counter() - t0)
    out["ns_value"] = None if v is None else float(v)
    out["exact"] = float(ev.clamp(min=0).sqrt().sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
