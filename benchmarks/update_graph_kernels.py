"""Replays the config #5 grouped update graph 50 times (for a rocprofv3 kernel trace of its nodes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NC, build  # noqa: E402
from torchmetrics_amd import MetricCollection  # noqa: E402
from torchmetrics_amd.utils.graphs import GraphedCompute, GraphedUpdate, UpdateGroup  # noqa: E402

dev = torch.device("cuda", 0)
cls, reg = build(dev)
g = torch.Generator().manual_seed(7)
lg = torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16)
lb = torch.randint(0, NC, (BATCH,), generator=g).to(dev)
x = torch.randn(BATCH, generator=g).to(dev)
y = x + 0.3 * torch.randn(BATCH, generator=g).to(dev)
cls_graph = MetricCollection({k: m for k, m in cls.items(keep_base=True) if k != "ece"}, compute_groups=True)
gu = GraphedUpdate(UpdateGroup((cls_graph, 2), (reg, 2)), lg, lb, x, y, bind_inputs=True)
cls["ece"].update(lg, lb)
gc = GraphedCompute(cls, reg)
torch.cuda.synchronize()
mark = torch.zeros(1, device=dev)
for i in range(50):
    mark.add_(1)  # step marker kernel
    gu()
    mark.add_(1)
    gc()
torch.cuda.synchronize()
print("done")
