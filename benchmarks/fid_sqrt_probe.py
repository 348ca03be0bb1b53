"""Probe: costs of the pieces of FID ``compute()`` and accuracy of a scaled Newton-Schulz trace-sqrt.

Times fp64 Cholesky, fp64 GEMM 2048^3 and the current eigvalsh path, then runs the scaled coupled Newton-Schulz
iteration on ``M = L^T Sigma2 L`` for well- and ill-conditioned covariances and reports the relative difference of
``tr sqrt(M)`` against eigvalsh.  One JSON line per measurement.
"""
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    return 1e3 * min(t)


def schedule(l0, tol=1e-15, extra=2):
    """Chen-Chow scale factors for s in [l0, 1] until the lower bound reaches 1."""
    alphas, l = [], l0
    while 1 - l > tol and len(alphas) < 100:
        a = math.sqrt(3.0 / (1.0 + l + l * l))
        alphas.append(a)
        l = a * l * (3 - a * a * l * l) / 2
    return alphas + [1.0] * extra


def ns_trace_sqrt(m, alphas, c=None, adaptive=False, rtol=1e-14, cap=80):
    """Scaled coupled Newton-Schulz: Y -> (m/c)^(1/2); T' = a (1.5 I - 0.5 a^2 Z Y) in one addmm, then Y T', T' Z.
    ``adaptive``: after the schedule keep iterating (a = 1) while tr Y still moves by more than ``rtol``."""
    d = m.shape[0]
    if c is None:
        c = m.diagonal().sum()
    eye = torch.eye(d, dtype=m.dtype, device=m.device)
    y = m / c
    z = eye.clone()
    prev = None
    k = 0
    seq = list(alphas)
    while True:
        a = seq[k] if k < len(seq) else 1.0
        t = torch.addmm(eye, z, y, beta=1.5 * a, alpha=-0.5 * a ** 3)
        y = y @ t
        z = t @ z
        k += 1
        if k >= len(seq):
            if not adaptive:
                break
            tr = float(y.diagonal().sum())
            if (prev is not None and abs(tr - prev) <= rtol * abs(tr)) or k >= cap:
                break
            prev = tr
    return c.sqrt() * y.diagonal().sum(), k


def main():
    dev = "cuda"
    d = 2048
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn(d, d, dtype=torch.float64, device=dev, generator=g)
    spd = a @ a.T / d + torch.eye(d, dtype=torch.float64, device=dev)
    print(json.dumps({"op": "potrf_2048_f64_ms", "v": timed(lambda: torch.linalg.cholesky_ex(spd))}), flush=True)
    print(json.dumps({"op": "gemm_2048_f64_ms", "v": timed(lambda: spd @ spd)}), flush=True)
    print(json.dumps({"op": "eigvalsh_2048_f64_ms", "v": timed(lambda: torch.linalg.eigvalsh(spd), reps=2)}),
          flush=True)
    n = 50_000
    for name, decay in (("random", 0.0), ("decay1e4", 4.0), ("decay1e8", 8.0)):
        scales = torch.logspace(0, -decay / 2, d, dtype=torch.float64, device=dev)
        f1 = torch.randn(n, d, dtype=torch.float64, device=dev, generator=g) * scales
        f2 = (torch.randn(n, d, dtype=torch.float64, device=dev, generator=g) * 1.1 + 0.05) * scales
        s1, s2 = torch.cov(f1.T), torch.cov(f2.T)
        del f1, f2
        lower = torch.linalg.cholesky(s1)
        m = lower.T @ s2 @ lower
        m = 0.5 * (m + m.T)
        ev = torch.linalg.eigvalsh(m)
        exact = ev.clamp(min=0).sqrt().sum()
        cond = float(ev.max() / ev.clamp(min=1e-300).min())
        p = s1 @ s2
        bounds = {"trace": p.diagonal().sum(), "min_norm": torch.minimum(torch.minimum(p.diagonal().sum(),
                  p.abs().sum(1).max()), p.abs().sum(0).max())}
        for form, mat in (("sym", m), ("nonsym", p)):
            for bname, cb in bounds.items():
                for l0, tol, extra, adaptive in ((1e-4, 1e-10, 1, False), (1e-5, 1e-10, 1, False),
                                                 (1e-4, 1e-10, 0, True), (1e-5, 1e-10, 0, True)):
                    al = schedule(l0, tol=tol, extra=extra)
                    v, k = ns_trace_sqrt(mat, al, c=cb,
                                         adaptive=adaptive)
                    ms = timed(lambda: ns_trace_sqrt(mat, al, c=cb, adaptive=adaptive), reps=2)
                    print(json.dumps({"case": name, "form": form, "bound": bname, "cond": cond, "l0": l0,
                                      "adaptive": adaptive, "iters": k, "ms": ms,
                                      "rel_err": float(((v - exact) / exact).abs())}), flush=True)


if __name__ == "__main__":
    main()
