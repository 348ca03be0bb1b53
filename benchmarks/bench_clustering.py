"""Clustering metrics at N = 10^7 labels (extrinsic) and 10^7 x 8 points (intrinsic): ours (``ops.contingency`` /
``cluster_sums`` / ``cluster_dispersion`` kernels) vs an op-for-op emulation of the reference paths
(``F/clustering/utils.py:119-173``: two ``unique(return_inverse)`` + sparse COO + ``to_dense``;
``F/clustering/davies_bouldin_score.py:46-57``: per-cluster boolean-mask loop).  One JSON line per case."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd.functional import clustering as F  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, out


def ref_contingency(preds, target):
    p_cls, p_idx = torch.unique(preds, return_inverse=True)
    t_cls, t_idx = torch.unique(target, return_inverse=True)
    coo = torch.sparse_coo_tensor(torch.stack((t_idx, p_idx)), torch.ones_like(p_idx),
                                  (t_cls.numel(), p_cls.numel()))
    return coo.coalesce().to_dense()


def ref_davies_bouldin(data, labels):
    uniq = torch.unique(labels)
    k = uniq.numel()
    cent = torch.zeros(k, data.shape[1], device=data.device, dtype=data.dtype)
    intra = torch.zeros(k, device=data.device, dtype=data.dtype)
    for i, lab in enumerate(uniq):
        ck = data[labels == lab]
        cent[i] = ck.mean(0)
        intra[i] = (ck - cent[i]).pow(2).sum(1).sqrt().mean()
    cd = torch.cdist(cent, cent)
    cd[cd == 0] = float("inf")
    return ((intra[None] + intra[:, None]) / cd).max(1).values.mean()


def main():
    # --ours-only: skip the emulated reference (its sparse COO / per-cluster ATen kernels) for an attributable trace
    ours_only = "--ours-only" in sys.argv[1:]
    dev = torch.device("cuda")
    n = 10_000_000
    g = torch.Generator(device=dev).manual_seed(0)
    t = torch.randint(0, 20, (n,), device=dev, generator=g)
    p = torch.where(torch.rand(n, device=dev, generator=g) < 0.7, (t * 7 + 3) % 25,
                    torch.randint(0, 25, (n,), device=dev, generator=g))
    ms_o, c_o = timed(lambda: F.calculate_contingency_matrix(p, t))
    if not ours_only:
        ms_r, c_r = timed(lambda: ref_contingency(p, t))
        assert torch.equal(c_o, c_r)
    else:
        ms_r = float("nan")
    print(json.dumps({"case": "contingency_1e7", "ours_ms": round(ms_o, 3), "reference_emulated_ms": round(ms_r, 3),
                      "speedup": round(ms_r / ms_o, 2)}), flush=True)
    ms_o, v_o = timed(lambda: F.adjusted_mutual_info_score(p, t))
    print(json.dumps({"case": "adjusted_mutual_info_1e7", "ours_ms": round(ms_o, 3), "value": float(v_o)}), flush=True)
    k, d = 17, 8
    centers = torch.randn(k, d, device=dev, generator=g) * 4
    labels = torch.randint(0, k, (n,), device=dev, generator=g)
    data = centers[labels] + torch.randn(n, d, device=dev, generator=g)
    ms_o, v_o = timed(lambda: F.davies_bouldin_score(data, labels))
    ms_r, v_r = timed(lambda: ref_davies_bouldin(data, labels), reps=2) if not ours_only else (float("nan"), v_o)
    print(json.dumps({"case": "davies_bouldin_1e7x8", "ours_ms": round(ms_o, 3), "reference_emulated_ms": round(ms_r, 3),
                      "speedup": round(ms_r / ms_o, 2), "rel_diff": abs(float(v_o) - float(v_r)) / abs(float(v_r))}),
          flush=True)
    ms_o, v_o = timed(lambda: F.calinski_harabasz_score(data, labels))
    print(json.dumps({"case": "calinski_harabasz_1e7x8", "ours_ms": round(ms_o, 3)}), flush=True)
    ms_o, v_o = timed(lambda: F.dunn_index(data, labels))
    print(json.dumps({"case": "dunn_1e7x8", "ours_ms": round(ms_o, 3)}), flush=True)


if __name__ == "__main__":
    main()
