"""Few-class multiclass stat-score update throughput (``mc_fewbins_tile_kernel`` path of csrc/classification/stat_scores.hip):
back-to-back ``MulticlassAccuracy(C).update`` on 1 M x C bf16 logits + int64 targets, wall clock over 200 updates
(as ``bench_binary_stats.py``), and the HIP-event median of single updates.  One JSON line per case; the knobs
TM_AMD_FEWBINS_TILE / TM_AMD_FEWBINS_R / TM_AMD_FEWBINS_FUSED are read once per process."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchmetrics_amd as tm  # noqa: E402


def main() -> None:
    g = torch.Generator(device="cuda").manual_seed(0)
    classes = [int(c) for c in os.environ.get("CLASSES", "10").split(",")]
    n = int(os.environ.get("ROWS", str(1 << 20)))
    for C in classes:
        for name, make in (("acc", lambda: tm.MulticlassAccuracy(C)), ("confmat", lambda: tm.MulticlassConfusionMatrix(C))):
            m = make().cuda()
            p = torch.rand(n, C, device="cuda", generator=g).to(torch.bfloat16)
            t = torch.randint(0, C, (n,), device="cuda", generator=g)
            ref = make()
            ref.update(p.float().cpu(), t.cpu())
            for _ in range(5):
                m.update(p, t)
            torch.cuda.synchronize()
            reps = 200
            t0 = time.perf_counter()
            for _ in range(reps):
                m.update(p, t)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / reps * 1e6
            ts = []
            for _ in range(31):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                m.update(p, t)
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            ts.sort()
            # 5 + 200 + 31 updates of the same batch: the states equal 236 x one CPU update
            ok = True
            for k, v in ref.metric_state.items():
                mine = getattr(m, k)
                if isinstance(v, torch.Tensor) and v.dtype == torch.int64:
                    ok = ok and torch.equal(mine.cpu(), v * 236)
            nbytes = p.numel() * 2 + t.numel() * 8
            print(json.dumps({"C": C, "n": n, "kind": name, "tile": os.environ.get("TM_AMD_FEWBINS_TILE", "dflt"),
                              "R": os.environ.get("TM_AMD_FEWBINS_R", "dflt"),
                              "fused": os.environ.get("TM_AMD_FEWBINS_FUSED", "dflt"),
                              "update_us": round(wall, 2), "TBps": round(nbytes / wall / 1e6, 2),
                              "event_us_median": round(ts[15], 2), "exact": ok}), flush=True)


if __name__ == "__main__":
    main()
