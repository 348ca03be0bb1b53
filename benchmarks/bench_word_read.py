"""Cost of reading one int32 device word on the host after a kernel, three ways (for ``Metric._raise_device_errors``).

* ``item``: ``buf.item()`` (ATen: blocking device->host copy into pageable memory);
* ``pinned_copy``: ``host.copy_(buf, non_blocking=True)`` into a pinned tensor + stream synchronize;
* ``gather_words``: our one-block kernel stores the word into mapped pinned memory + stream synchronize.

Each read follows a 1000-class confusion-matrix update on 8192 bf16 rows (the headline's compute point), so the
numbers include waiting for real work.  Prints one JSON line per method: median / p10 / p90 wall microseconds.
"""
import json
import time

import torch

import torchmetrics_amd as tm
from torchmetrics_amd import ops


def main() -> None:
    dev = torch.device("cuda", 0)
    m = tm.MulticlassConfusionMatrix(1000).to(dev)
    p = torch.randn(8192, 1000, device=dev, dtype=torch.bfloat16)
    t = torch.randint(0, 1000, (8192,), device=dev)
    buf = torch.zeros(1, dtype=torch.int32, device=dev)
    host = torch.zeros(128, dtype=torch.int32, pin_memory=True)
    hptr = int(ops._ops().mapped_device_ptr(host))
    table = torch.tensor([[buf.data_ptr(), 0]], dtype=torch.int64)
    stream = torch.cuda.current_stream(dev)

    def item():
        return int(buf.item())

    def pinned_copy():
        host[:1].copy_(buf, non_blocking=True)
        stream.synchronize()
        return int(host[0])

    def gather_words():
        ops._ops().gather_words(table, hptr, buf)
        stream.synchronize()
        return int(host[0])

    def gather_words_table():  # the table built per call, as a metric without a cached table would
        tb = torch.tensor([[buf.data_ptr(), 0]], dtype=torch.int64)
        ops._ops().gather_words(tb, hptr, buf)
        stream.synchronize()
        return int(host[0])

    for name, fn in (("item", item), ("pinned_copy", pinned_copy), ("gather_words", gather_words),
                     ("gather_words_table", gather_words_table)):
        for _ in range(20):
            m.update(p, t)
            fn()
        wall, alone = [], []
        for _ in range(300):
            m.update(p, t)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            alone.append((time.perf_counter() - t0) * 1e6)
            m.update(p, t)
            t0 = time.perf_counter()
            fn()
            wall.append((time.perf_counter() - t0) * 1e6)
        wall.sort()
        alone.sort()
        print(json.dumps({"method": name, "idle_us_p50": round(alone[150], 2), "idle_us_p10": round(alone[30], 2),
                          "after_update_us_p50": round(wall[150], 2), "after_update_us_p10": round(wall[30], 2),
                          "after_update_us_p90": round(wall[270], 2)}), flush=True)


if __name__ == "__main__":
    main()
