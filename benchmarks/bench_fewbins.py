"""Few-class multiclass stat / confusion-matrix updates (mc_fewbins_tile_kernel, csrc/classification/stat_scores.hip):
kernel time (HIP events, median of 30) for several class counts and row counts; one JSON line per case.
Knobs: TM_AMD_FEWBINS_TILE (blocks per CU of the tiled kernel; 0 = the per-row staging kernel)."""
import json
import os

import torch

import torchmetrics_amd as tm


def main() -> None:
    g = torch.Generator(device="cuda").manual_seed(0)
    for C in (4, 10, 32):
        for n in (1 << 16, 1 << 20, 1 << 22):
            for name, m in (("acc", tm.MulticlassAccuracy(C)), ("confmat", tm.MulticlassConfusionMatrix(C))):
                m = m.cuda()
                p = torch.rand(n, C, device="cuda", generator=g).to(torch.bfloat16)
                t = torch.randint(0, C, (n,), device="cuda", generator=g)
                for _ in range(3):
                    m.update(p, t)
                ts = []
                for _ in range(30):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    m.update(p, t)
                    b.record()
                    b.synchronize()
                    ts.append(a.elapsed_time(b) * 1e3)
                ts.sort()
                us = ts[15]
                gb = (p.numel() * 2 + t.numel() * 8) / 1e9
                print(json.dumps({"tile": os.environ.get("TM_AMD_FEWBINS_TILE", "2"), "C": C, "n": n, "kind": name,
                                  "us": round(us, 2), "TBps": round(gb / us * 1e6 / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
