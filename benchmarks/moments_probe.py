"""Per-launch time of the moments kernels (``csrc/regression/moments.hip``) against batch size and requested sums:
back-to-back launches timed with events (each call is kernel-bound above ~6 us).  Cases: one sum (SSE), the config #5
regression collection's merged request (MSE / MAE / R2 / EV sums + the Pearson fold), and the fold alone."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd import ops  # noqa: E402


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="*", default=[1024, 4096, 8192, 16384, 32768, 65536])
    ap.add_argument("--cases", nargs="*", default=["sse", "config5", "fold_only"])
    args = ap.parse_args()
    dev = torch.device("cuda")
    for n in args.n:
        g = torch.Generator(device=dev).manual_seed(n)
        x = torch.randn(n, device=dev, generator=g)
        y = x + 0.3 * torch.randn(n, device=dev, generator=g)
        plain = [torch.zeros(1, device=dev, dtype=torch.float32) for _ in range(12)]
        fold = [torch.zeros(1, device=dev, dtype=torch.float32) for _ in range(6)]
        sp, st = fold[0], fold[1]
        cases = {
            "sse": lambda: ops.moments_update(x, y, 1, [], plain[:1], [ops.SSE]),
            "config5": lambda: ops.moments_update(
                x, y, 1, [], fold + plain[:8],
                [ops.SSE, ops.COUNT, ops.SAE, ops.COUNT, ops.sum_diff(ops.ST, ops.SP), ops.SSE, ops.ST, ops.STT],
                shift_p=sp, shift_t=st, fold=ops.FOLD_PEARSON),
            "fold_only": lambda: ops.moments_update(x, y, 1, [], fold, [], shift_p=sp, shift_t=st,
                                                    fold=ops.FOLD_PEARSON),
        }
        row = {"n": n}
        for name, fn in cases.items():
            if name not in args.cases:
                continue
            for _ in range(20):
                fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            for _ in range(200):
                fn()
            b.record()
            torch.cuda.synchronize()
            row[name + "_us"] = round(a.elapsed_time(b) * 1e3 / 200, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
