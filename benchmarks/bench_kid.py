"""KID compute (50k x 2048 features per distribution, 100 subsets of 1000) and MiFID's cosine distance vs the
reference's formulations (S/image/kid.py:255-276: host randperm + 3 GEMMs + pow + sums per subset in a Python loop;
S/image/mifid.py:36-63: normalise, mm, abs, row min) on the same device."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd.image import KernelInceptionDistance  # noqa: E402
from torchmetrics_amd.image.generative import _compute_cosine_distance  # noqa: E402


class _Id(torch.nn.Module):
    def __init__(self, d):
        super().__init__()
        self.num_features = d

    def forward(self, x):
        return x


def ref_kid(real, fake, subsets=100, m=1000, degree=3, coef=1.0):
    gamma = 1.0 / real.shape[1]
    scores = []
    for _ in range(subsets):
        fr = real[torch.randperm(real.shape[0])[:m]]
        ff = fake[torch.randperm(fake.shape[0])[:m]]
        k11 = (fr @ fr.T * gamma + coef) ** degree
        k22 = (ff @ ff.T * gamma + coef) ** degree
        k12 = (fr @ ff.T * gamma + coef) ** degree
        v = ((k11.sum(-1) - torch.diag(k11)).sum() + (k22.sum(-1) - torch.diag(k22)).sum()) / (m * (m - 1))
        scores.append(v - 2 * k12.sum(0).sum() / m**2)
    s = torch.stack(scores)
    return s.mean(), s.std(unbiased=False)


def ref_cos(f1, f2):
    n1 = f1 / torch.norm(f1, dim=1, keepdim=True)
    n2 = f2 / torch.norm(f2, dim=1, keepdim=True)
    return torch.mean((1.0 - torch.abs(n1 @ n2.t())).min(dim=1).values)


def timeit(fn, iters=3):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    n, d = 50000, 2048
    real = torch.randn(n, d, device=dev, generator=g)
    fake = torch.randn(n, d, device=dev, generator=g) + 0.05
    kid = KernelInceptionDistance(feature=_Id(d)).to(dev)
    kid.update(real, True)
    kid.update(fake, False)

    def ours():
        kid._computed = None
        return kid.compute()

    a, b = ours(), ref_kid(real, fake)
    print(json.dumps({"case": "kid compute 50k x 2048, 100 x 1000", "ours_ms": round(timeit(ours), 3),
                      "ref_ms": round(timeit(lambda: ref_kid(real, fake), 1), 3),
                      "kid_ours": float(a[0]), "kid_ref": float(b[0]),
                      "note": "different (equally distributed) subset draws: values agree statistically"}), flush=True)
    f1, f2 = real[:20000], fake[:20000]
    o, r = _compute_cosine_distance(f1, f2, 10.0), ref_cos(f1, f2)
    print(json.dumps({"case": "mifid cosine distance 20k x 20k x 2048", "ours_ms": round(timeit(
        lambda: _compute_cosine_distance(f1, f2, 10.0)), 3), "ref_ms": round(timeit(lambda: ref_cos(f1, f2)), 3),
        "abs_diff": abs(float(o) - float(r))}), flush=True)


if __name__ == "__main__":
    main()
