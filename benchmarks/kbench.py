"""Kernel-level timing (HIP events, many reps, interleaved A/B in one process) for the hot ops.

Usage: ``python benchmarks/kbench.py [--only NAME]``; prints one JSON line per case.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd import ops  # noqa: E402


def timeit(fn, reps: int = 200, warmup: int = 20) -> float:
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    for _ in range(reps):
        fn()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) / reps * 1e3  # us


def case_confmat(N=8192, C=1000, dtype=torch.bfloat16):
    dev = "cuda"
    nbuf = 4  # cycle buffers like bench.py (inputs not L2-resident, as in a real eval loop)
    preds_l = [torch.randn(N, C, device=dev).to(dtype) for _ in range(nbuf)]
    target_l = [torch.randint(0, C, (N,), device=dev) for _ in range(nbuf)]
    preds = preds_l[0]
    cm = torch.zeros(C * C, dtype=torch.int64, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    it = [0]

    def ours():
        i = it[0] = (it[0] + 1) % nbuf
        ops.mc_update(preds_l[i], target_l[i], cm, flag, C, None, ops.MC_CONFMAT, False)

    def aten():
        i = it[0] = (it[0] + 1) % nbuf
        lab = preds_l[i].argmax(1)
        cm.add_(torch.bincount(target_l[i] * C + lab, minlength=C * C))

    t_ours = timeit(ours)
    t_aten = timeit(aten)
    gbps = preds.numel() * preds.element_size() / (t_ours * 1e-6) / 1e9
    return {"case": f"confmat N={N} C={C} {dtype}", "ours_us": round(t_ours, 2), "aten_us": round(t_aten, 2),
            "ours_GBps": round(gbps, 1)}


def case_binary(N=1 << 22, dtype=torch.float32):
    dev = "cuda"
    preds = torch.rand(N, device=dev).to(dtype)
    target = torch.randint(0, 2, (N,), device=dev)
    ws = torch.zeros(7, dtype=torch.int64, device=dev)
    np_ = torch.zeros(1, dtype=torch.int32, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    outs = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(4)]

    def ours():
        ops.bin_update(preds, target, ws, flag, np_, 1, 0.5, None, False)
        ops.bin_stats_finalize(ws, np_, True, *outs)

    def aten():
        p = preds
        if not torch.all((p >= 0) * (p <= 1)):
            p = p.sigmoid()
        p = p > 0.5
        tp = ((target == p) & (target == 1)).sum()
        fn = ((target != p) & (target == 1)).sum()
        fp = ((target != p) & (target == 0)).sum()
        tn = ((target == p) & (target == 0)).sum()
        return tp, fp, tn, fn

    t_ours, t_aten = timeit(ours), timeit(aten)
    return {"case": f"binary stat N={N} {dtype}", "ours_us": round(t_ours, 2), "aten_us": round(t_aten, 2)}


CASES = {"confmat": case_confmat, "binary": case_binary}

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--N", type=int, default=0)
    ap.add_argument("--C", type=int, default=0)
    a = ap.parse_args()
    if a.N:
        print(json.dumps(case_confmat(N=a.N, C=a.C)))
        sys.exit(0)
    for name, fn in CASES.items():
        if a.only and a.only != name:
            continue
        print(json.dumps(fn()))
        if name == "confmat":
            print(json.dumps(fn(N=65536, C=1000)))
            print(json.dumps(fn(N=8192, C=32000)))
            print(json.dumps(fn(N=8192, C=10, dtype=torch.float32)))
