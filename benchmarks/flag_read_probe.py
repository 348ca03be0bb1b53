"""Cost of reading a device int32 flag word on the host (the compute()-time validation check), by method."""
import json
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return 1e6 * (time.perf_counter() - t0) / reps


def main():
    dev = torch.device("cuda")
    buf = torch.zeros(1, dtype=torch.int32, device=dev)
    pinned = torch.zeros(1, dtype=torch.int32).pin_memory()
    stream = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    x = torch.zeros(1, device=dev)

    def item():
        return int(buf.item())

    def pinned_stream_sync():
        pinned.copy_(buf, non_blocking=True)
        stream.synchronize()
        return int(pinned[0])

    def pinned_event_sync():
        pinned.copy_(buf, non_blocking=True)
        ev.record(stream)
        ev.synchronize()
        return int(pinned[0])

    def numpy_view():
        pinned.copy_(buf, non_blocking=True)
        stream.synchronize()
        return int(pinned.numpy()[0])

    def stream_sync_only():
        stream.synchronize()

    def tiny_kernel():
        x.add_(1)

    out = {k: timed(f) for k, f in (("item", item), ("pinned_stream_sync", pinned_stream_sync),
                                      ("pinned_event_sync", pinned_event_sync), ("pinned_numpy", numpy_view),
                                      ("stream_sync_idle", stream_sync_only), ("tiny_kernel_launch", tiny_kernel))}
    torch.cuda.synchronize()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
