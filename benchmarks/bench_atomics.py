"""Device-scope atomic flush cost on MI355X (csrc/common/probes.hip): `blocks` blocks each add into the same `bins`
histogram addresses (the few-bin kernels' per-block flush), int32 / int64, bins adjacent or 256 B apart.
Prints one JSON line per case: kernel time from HIP events (median of 50)."""
import json

import torch

from torchmetrics_amd import ops


def main() -> None:
    op = ops._ops().atomic_probe
    for dtype in (torch.int64, torch.int32):
        for bins, spread in ((1, 1), (31, 1), (31, 64)):
            for blocks in (1, 64, 256, 512, 1024, 4096):
                out = torch.zeros(bins * spread + 1, dtype=dtype, device="cuda")
                for _ in range(3):
                    op(out, blocks, bins, spread)
                times = []
                for _ in range(50):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    op(out, blocks, bins, spread)
                    b.record()
                    b.synchronize()
                    times.append(a.elapsed_time(b) * 1e3)
                times.sort()
                print(json.dumps({"dtype": str(dtype).replace("torch.", ""), "bins": bins, "spread": spread,
                                  "blocks": blocks, "us": round(times[25], 2)}), flush=True)


if __name__ == "__main__":
    main()
