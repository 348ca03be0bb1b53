"""Round-2 kernels vs the op chains they replace (same inputs, same process): multilabel ranking rows, BERTScore
greedy matching (GEMM row/column-max epilogue), device RLE encode, many-output regression moments.
One JSON line per case: ours_ms, torch_ms (the previous / reference-shaped op chain), speedup, max |diff|."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd import ops  # noqa: E402
from torchmetrics_amd.functional.classification import ranking as RK  # noqa: E402
from torchmetrics_amd.functional.text import bert as BT  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        out = fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / reps, out


def without_kernel(fn, *args):
    saved = ops.label_ranking_rows
    ops.label_ranking_rows = lambda *a, **k: None
    try:
        return fn(*args)
    finally:
        ops.label_ranking_rows = saved


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    preds = torch.rand(100_000, 64, device=dev, generator=g)
    target = torch.randint(0, 2, (100_000, 64), device=dev, generator=g)
    for name, fn in (("coverage", RK._multilabel_coverage_error_update),
                     ("lrap", RK._multilabel_ranking_average_precision_update),
                     ("ranking_loss", RK._multilabel_ranking_loss_update)):
        t_ours, a = timed(lambda: fn(preds, target))
        t_ref, b = timed(lambda: without_kernel(fn, preds, target))
        print(json.dumps({"case": f"multilabel_{name} 1e5x64", "ours_ms": round(t_ours, 4), "torch_ms": round(t_ref, 4),
                          "speedup": round(t_ref / t_ours, 2),
                          "abs_diff": float((a[0].double() - b[0].double()).abs())}), flush=True)

    n, p, r, d = 256, 512, 512, 768
    pe = torch.nn.functional.normalize(torch.randn(n, 1, p, d, device=dev, generator=g), dim=-1)
    te = torch.nn.functional.normalize(torch.randn(n, 1, r, d, device=dev, generator=g), dim=-1)
    pw, tw = torch.rand(n, p, device=dev, generator=g), torch.rand(n, r, device=dev, generator=g)

    def torch_match():
        cos = torch.matmul(pe, te.transpose(-1, -2))
        return (cos.amax(dim=3) * pw[:, None]).sum(-1), (cos.amax(dim=2) * tw[:, None]).sum(-1)

    t_ours, a = timed(lambda: BT._greedy_match(pe, te, pw, tw))
    t_ref, b = timed(torch_match)
    print(json.dumps({"case": "bertscore_greedy_match 256 pairs x 512x512 tokens x 768", "ours_ms": round(t_ours, 4),
                      "torch_ms": round(t_ref, 4), "speedup": round(t_ref / t_ours, 2),
                      "abs_diff": float((a[0] - b[0]).abs().max())}), flush=True)

    masks = [(torch.rand(100, 480, 640, device=dev, generator=g) < 0.0) for _ in range(8)]
    yy = torch.arange(480, device=dev).view(1, 480, 1)
    xx = torch.arange(640, device=dev).view(1, 1, 640)
    for i in range(8):
        c = torch.randint(50, 400, (100, 2), device=dev, generator=g)
        masks[i] = ((yy - c[:, 0].view(-1, 1, 1)).abs() < 40) & ((xx - c[:, 1].view(-1, 1, 1)).abs() < 60)
    t_ours, packs = timed(lambda: ops.rle_encode(masks), reps=10)
    nbytes = sum(m.numel() for m in masks)
    print(json.dumps({"case": "rle_encode 8 images x 100 masks @ 640x480", "ours_ms": round(t_ours, 4),
                      "input_GBps": round(nbytes / t_ours / 1e6, 1),
                      "pack_MB": round(sum(p.numel() * 4 for p in packs) / 2**20, 3),
                      "dense_MB": round(nbytes / 2**20, 1)}), flush=True)

    k = 4096
    x = torch.randn(20_000, k, device=dev, generator=g)
    y = x + torch.randn(20_000, k, device=dev, generator=g)
    out = torch.zeros(k, device=dev)
    t_ours, _ = timed(lambda: ops.moments_update(x, y, k, [], [out], [ops.SSE]))
    t_ref, _ = timed(lambda: out.add_(((x - y) ** 2).sum(0)))
    print(json.dumps({"case": "moments sse 2e4 x 4096 outputs", "ours_ms": round(t_ours, 4), "torch_ms": round(t_ref, 4),
                      "speedup": round(t_ref / t_ours, 2),
                      "GBps": round(2 * x.numel() * 4 / t_ours / 1e6, 1)}), flush=True)
    del x, y

    from torchmetrics_amd.classification import MulticlassAccuracy

    for dtype in (torch.bfloat16, torch.float32):
        s = torch.randn(65536, 1000, device=dev, generator=g).to(dtype)
        lab = torch.randint(0, 1000, (65536,), device=dev, generator=g)
        t_ours, a = timed(lambda: ops.topk_labels(s, 5))
        t_ref, b = timed(lambda: torch.topk(s, 5, dim=1).indices)
        print(json.dumps({"case": f"topk_labels k=5 65536x1000 {str(dtype)[6:]}", "ours_ms": round(t_ours, 4),
                          "torch_ms": round(t_ref, 4), "speedup": round(t_ref / t_ours, 2),
                          "GBps": round(s.numel() * s.element_size() / t_ours / 1e6, 1),
                          "mismatch_rows": int((a.long() != b).any(1).sum())}), flush=True)
        m = MulticlassAccuracy(num_classes=1000, top_k=5).to(dev)
        t_ours, _ = timed(lambda: m.update(s, lab))
        saved = ops.mc_topk_update
        ops.mc_topk_update = lambda *a, **k: False  # torch.topk labels + the label histogram kernel
        try:
            t_ref, _ = timed(lambda: m.update(s, lab))
        finally:
            ops.mc_topk_update = saved
        print(json.dumps({"case": f"MulticlassAccuracy(top_k=5).update 65536x1000 {str(dtype)[6:]}",
                          "ours_ms": round(t_ours, 4), "torch_topk_ms": round(t_ref, 4),
                          "speedup": round(t_ref / t_ours, 2)}), flush=True)


if __name__ == "__main__":
    main()
