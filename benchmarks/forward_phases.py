"""Host time per phase of ``Metric.forward`` (reduce-state path) on ROCm: batch reset, update, batch compute, merge.
Median over 300 calls, in microseconds; one JSON line per metric."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchmetrics_amd as tm  # noqa: E402
from torchmetrics_amd.metric import Metric  # noqa: E402


def phases(m, preds, target, n=300):
    rec = {"reset": [], "update": [], "compute": [], "merge": [], "total": []}
    for i in range(n + 20):
        t0 = time.perf_counter()
        global_state = {attr: getattr(m, attr) for attr in m._defaults}
        count = m._update_count
        saved = m._enter_batch_mode()
        m._batch_reset()
        t1 = time.perf_counter()
        m.update(preds, target)
        t2 = time.perf_counter()
        val = m.compute()
        t3 = time.perf_counter()
        m._update_count = count + 1
        with torch.no_grad():
            if m._inplace_forward_merge:
                m._merge_sums_in_place(global_state)
            m._reduce_states(global_state)
        m._exit_batch_mode(saved)
        t4 = time.perf_counter()
        if i >= 20:
            for k, a, b in (("reset", t0, t1), ("update", t1, t2), ("compute", t2, t3), ("merge", t3, t4),
                            ("total", t0, t4)):
                rec[k].append((b - a) * 1e6)
        del val
    torch.cuda.synchronize()
    return {k: round(statistics.median(v), 1) for k, v in rec.items()}


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    preds = torch.randn(8192, 1000, device="cuda", generator=g).to(torch.bfloat16)
    target = torch.randint(0, 1000, (8192,), device="cuda", generator=g)
    for name, make in (("MulticlassAccuracy(1000)", lambda: tm.MulticlassAccuracy(1000)),
                       ("MulticlassConfusionMatrix(1000)", lambda: tm.MulticlassConfusionMatrix(1000))):
        m = make().cuda()
        for _ in range(10):
            m(preds, target)
        torch.cuda.synchronize()
        print(json.dumps({"metric": name, **phases(m, preds, target)}), flush=True)


if __name__ == "__main__":
    main()
