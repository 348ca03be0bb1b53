"""Config #5 classification collection update only (the fused family update, utils/fused_update.py), 300 steps,
for counter / ablation runs of family_rows_g_kernel (TM_AMD_FAMILY_ABLATE, TM_AMD_FAMILY_G, TM_AMD_FAMILY_BLOCKS).
Prints the mean step time from events."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NC, build  # noqa: E402


def main() -> None:
    dev = torch.device("cuda")
    cls, _ = build(dev)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16)
    y = torch.randint(0, NC, (BATCH,), generator=g).to(dev)
    for _ in range(20):
        cls.update(x, y)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(300):
        cls.update(x, y)
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"ablate": os.environ.get("TM_AMD_FAMILY_ABLATE", "0"), "G": os.environ.get("TM_AMD_FAMILY_G", "1"),
                      "step_us": round(a.elapsed_time(b) * 1e3 / 300, 2)}), flush=True)


if __name__ == "__main__":
    main()
