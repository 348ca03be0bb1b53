"""BASELINE config #4: FrechetInceptionDistance on random 50k x 2048 feature tensors (real + fake), 1 -> N ranks.

Strong scaling: the 50k real + 50k fake features are split over the ranks (rank r updates every W-th batch); each
rank accumulates Σx / XᵀX on its device (fp64-MFMA SYRK), then ``compute()`` syncs the states -- f64[D] sums, f64[D,D]
covariance sums, sample counts: two 32 MiB all-reduces over RCCL at D = 2048 -- and evaluates the FID (Newton-Schulz
on our fp64 GEMM).  The in-run baseline is an op-for-op emulation of the reference (``S/image/fid.py:332-361``:
``features.double()``, ``sum(0)``, ``t().mm()`` per batch; sync per state tensor with barrier + all_gather(shape) +
all_gather(data) + stack + sum (``S/utilities/distributed.py:97-147``); compute with ``torch.linalg.eigvals``).

Also reported: the fp64 FID before the cast to the feature dtype, against a symmetric eigensolve of the same synced
covariances (``rel_diff_fp64_vs_eigh``) -- the returned float32 value's own rounding is ~3e-8.

Usage: ``python benchmarks/bench_fid.py [--samples 50000 --dim 2048 --batch 1000]``; N ranks: under torch.distributed.run.
Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks._dist import barrier_sync, dist_info, launch, max_over_ranks, setup, sync, teardown  # noqa: E402
from torchmetrics_amd.image import FrechetInceptionDistance  # noqa: E402
from torchmetrics_amd.image.generative import _compute_fid  # noqa: E402
from torchmetrics_amd.parallel.sync import comm_stats  # noqa: E402


class _Id(torch.nn.Module):
    def __init__(self, d: int) -> None:
        super().__init__()
        self.num_features = d

    def forward(self, x):
        return x


def ours(real, fake, d, device, world):
    m = FrechetInceptionDistance(feature=_Id(d)).to(device)
    barrier_sync(device, world)
    t0 = time.perf_counter()
    for r, f in zip(real, fake):
        m.update(r, real=True)
        m.update(f, real=False)
    barrier_sync(device, world)
    t1 = time.perf_counter()
    v = m.compute()
    barrier_sync(device, world)
    t2 = time.perf_counter()
    return m, float(v), t1 - t0, t2 - t1


def _gather_all_tensors(t):
    """The reference's per-state gather: barrier, all_gather of the shape, all_gather of the data."""
    t = t.contiguous()
    w = dist.get_world_size()
    dist.barrier()
    shape = torch.tensor(t.shape, device=t.device)
    shapes = [torch.zeros_like(shape) for _ in range(w)]
    dist.all_gather(shapes, shape)
    out = [torch.zeros_like(t) for _ in range(w)]
    dist.all_gather(out, t)
    return out


def reference(real, fake, n_total, d, device, world):
    st = {k: torch.zeros(d, dtype=torch.float64, device=device) for k in ("rs", "fs")}
    cv = {k: torch.zeros(d, d, dtype=torch.float64, device=device) for k in ("rc", "fc")}
    barrier_sync(device, world)
    t0 = time.perf_counter()
    for r, f in zip(real, fake):
        rd, fd = r.double(), f.double()
        st["rs"] += rd.sum(0)
        cv["rc"] += rd.t().mm(rd)
        st["fs"] += fd.sum(0)
        cv["fc"] += fd.t().mm(fd)
    barrier_sync(device, world)
    t1 = time.perf_counter()
    if world > 1:
        for dct in (st, cv):
            for k in dct:
                dct[k] = torch.stack(_gather_all_tensors(dct[k])).sum(0)
        for _ in range(2):  # the two num_samples states
            _gather_all_tensors(torch.tensor(n_total // world, device=device))
    n = n_total
    mr, mf = (st["rs"] / n).unsqueeze(0), (st["fs"] / n).unsqueeze(0)
    cr = (cv["rc"] - n * mr.t().mm(mr)) / (n - 1)
    cf = (cv["fc"] - n * mf.t().mm(mf)) / (n - 1)
    a = (mr - mf).square().sum()
    b = cr.trace() + cf.trace()
    c = torch.linalg.eigvals(cr @ cf).sqrt().real.sum(dim=-1)
    v = a + b - 2 * c
    sync(device)
    barrier_sync(device, world)
    t2 = time.perf_counter()
    return float(v), t1 - t0, t2 - t1


def fp64_check(m):
    """fp64 FID of the synced states: our compute path vs a symmetric eigensolve (Cholesky similarity)."""
    with m.sync_context(should_unsync=True):
        n_r, n_f = m.real_features_num_samples, m.fake_features_num_samples
        mr, mf = m.real_features_sum / n_r, m.fake_features_sum / n_f
        cr = (m.real_features_cov_sum - n_r * torch.outer(mr, mr)) / (n_r - 1)
        cf = (m.fake_features_cov_sum - n_f * torch.outer(mf, mf)) / (n_f - 1)
        ours64 = float(_compute_fid(mr, cr, mf, cf))
        lower = torch.linalg.cholesky(cr)
        mm = lower.T @ cf @ lower
        tr = torch.linalg.eigvalsh(0.5 * (mm + mm.T)).clamp(min=0).sqrt().sum()
        eigh64 = float((mr - mf).square().sum() + cr.trace() + cf.trace() - 2 * tr)
    return ours64, eigh64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks to run (default: WORLD_SIZE or 1); N > 1 without a "
                    "launcher spawns N ranks itself")
    ap.add_argument("--samples", type=int, default=50_000)
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=1000)
    ap.add_argument("--no-baseline", action="store_true")
    ap.add_argument("--ours-only", action="store_true",
                    help="only this package's update + compute (no emulated reference, no eigensolve parity check): "
                         "for an attributable kernel trace")
    args = ap.parse_args()
    launch(args.gpus or int(os.environ.get("WORLD_SIZE", "1")), __file__)
    world, rank, device = setup()
    nb = args.samples // args.batch
    g = torch.Generator(device=device).manual_seed(0)
    real_all = [torch.randn(args.batch, args.dim, device=device, generator=g) for _ in range(nb)]
    fake_all = [torch.randn(args.batch, args.dim, device=device, generator=g) * 1.1 + 0.05 for _ in range(nb)]
    real, fake = real_all[rank::world], fake_all[rank::world]  # this rank's share (identical data on every rank)
    ours(real[:1], fake[:1], args.dim, device, world)  # warm-up (kernels, allocator, communicators)
    comm_stats(reset=True)
    m, v_o, up_o, cp_o = ours(real, fake, args.dim, device, world)
    comms = dist_info(world)
    up_o, cp_o = max_over_ranks(up_o, device, world), max_over_ranks(cp_o, device, world)
    ours64 = eigh64 = None
    if not args.ours_only:
        ours64, eigh64 = fp64_check(m)
    base = None
    if not args.no_baseline and not args.ours_only:
        v_r, up_r, cp_r = reference(real, fake, nb * args.batch, args.dim, device, world)
        up_r, cp_r = max_over_ranks(up_r, device, world), max_over_ranks(cp_r, device, world)
        base = {"fid": v_r, "update_s": round(up_r, 4), "compute_s": round(cp_r, 4),
                "features_per_s": round(2 * args.samples / up_r, 1), "rel_diff_vs_ours": abs(v_o - v_r) / max(abs(v_r), 1e-12)}
    if rank == 0:
        out = {
            "metric": f"FID update features/s and synced compute wall-clock ({args.samples} x {args.dim} real + fake)",
            "n_gpus": world,
            "scaling": "strong",
            "ours": {"fid": v_o, "update_s": round(up_o, 4), "compute_s": round(cp_o, 4),
                     "features_per_s": round(2 * args.samples / up_o, 1)},
            "reference_emulated": base,
            "update_plus_compute_s": {"ours": round(up_o + cp_o, 4),
                                      "reference_emulated": round(base["update_s"] + base["compute_s"], 4) if base else None},
            "end_to_end_speedup": round((base["update_s"] + base["compute_s"]) / (up_o + cp_o), 3) if base else None,
            "compute_speedup": round(base["compute_s"] / cp_o, 3) if base else None,
            "fid_fp64": ours64,
            "fid_fp64_eigh": eigh64,
            "rel_diff_fp64_vs_eigh": abs(ours64 - eigh64) / max(abs(eigh64), 1e-12) if eigh64 is not None else None,
            "dist": comms,
            "device": torch.cuda.get_device_name(device) if device.type == "cuda" else "cpu",
        }
        print(json.dumps(out), flush=True)
    teardown(world)


if __name__ == "__main__":
    main()
