"""Host-side cost per ``update`` (tiny inputs so the GPU is never the bottleneck)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchmetrics_amd as tm  # noqa: E402
from torchmetrics_amd import ops  # noqa: E402


def rate(fn, n=3000):
    for _ in range(100):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6


def main():
    ops.load_native()
    dev = "cuda"
    C = 1000
    preds = torch.randn(64, C, device=dev, dtype=torch.bfloat16)
    target = torch.randint(0, C, (64,), device=dev)
    cm = torch.zeros(C * C, dtype=torch.int64, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    m = tm.MulticlassConfusionMatrix(C).to(dev)
    from torchmetrics_amd.functional.classification.confusion_matrix import (
        _multiclass_confusion_matrix_tensor_validation as _val,
    )

    class _Noop(tm.Metric):
        full_state_update = False

        def update(self, p, t):
            pass

        def compute(self):
            return 0

    noop = _Noop().to(dev)
    m2 = tm.MulticlassConfusionMatrix(C, validate_args=False).to(dev)
    acc = tm.MulticlassAccuracy(C).to(dev)
    res = {
        "raw_torch_ops_call_us": rate(lambda: torch.ops.tm_amd.mc_update(preds, target, cm, flag, C, 0, False, 0, False)),
        "raw_fastcall_us": rate(lambda: ops._fast_mod.mc_update(preds, target, cm, flag, C, 0, False, 0, False)),
        "fastcall_args_only_us": rate(lambda: ops._fast_mod.arg_probe(preds, target, cm, flag, C, 0, False, 0, False)),
        "fastcall_empty_launch_us": rate(lambda: ops._fast_mod.launch_probe(flag)),
        "validation_only_us": rate(lambda: _val(preds, target, C, None)),
        "preds.device_us": rate(lambda: preds.device),
        "wrapper_noop_update_us": rate(lambda: noop.update(preds, target)),
        "ops.mc_update_us": rate(lambda: ops.mc_update(preds, target, cm, flag, C, None, 0, False)),
        "MulticlassConfusionMatrix.update_us": rate(lambda: m.update(preds, target)),
        "MulticlassConfusionMatrix(validate_args=False).update_us": rate(lambda: m2.update(preds, target)),
        "MulticlassAccuracy.update_us": rate(lambda: acc.update(preds, target)),
        "empty_torch_add_us": rate(lambda: flag.add_(0)),
    }
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
