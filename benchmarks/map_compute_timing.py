"""Config #3's ``MeanAveragePrecision.compute()`` alone (512 images x 100 detections, COCO-80, class metrics): the
median / min wall-clock of 30 computes of the same states, for the shipped path and for the round-6-start variant
whose configuration constants and image sizes crossed to the device with synchronous (stream-draining) host copies.
One JSON line per variant."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_map import make_data  # noqa: E402
from torchmetrics_amd.detection import MeanAveragePrecision  # noqa: E402
from torchmetrics_amd.detection import _coco_eval  # noqa: E402


def _sync_const(values, dev):
    return torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev)


def _sync_sizes(values, dev):
    return torch.tensor(values, dtype=torch.long).to(dev, non_blocking=True)


def timed(m, reps=30):
    out = []
    for _ in range(reps):
        m._computed = None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.compute()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
    return out


def main():
    dev = torch.device("cuda", 0)
    preds, target = make_data(512, dev)
    m = MeanAveragePrecision(class_metrics=True).to(dev)
    for i in range(0, 512, 64):
        m.update(preds[i:i + 64], target[i:i + 64])
    shipped = (_coco_eval._device_const, _coco_eval._to_device_async)
    for _ in range(3):
        m._computed = None
        m.compute()
    for variant in ("shipped", "sync_copies", "shipped", "sync_copies"):
        if variant == "shipped":
            _coco_eval._device_const, _coco_eval._to_device_async = shipped
        else:
            _coco_eval._device_const, _coco_eval._to_device_async = _sync_const, _sync_sizes
        ts = timed(m)
        print(json.dumps({"variant": variant, "compute_ms_median": round(statistics.median(ts), 3),
                          "compute_ms_min": round(min(ts), 3), "reps": len(ts)}), flush=True)
    _coco_eval._device_const, _coco_eval._to_device_async = shipped


if __name__ == "__main__":
    main()
