"""One few-class case for counter collection / kernel traces: MulticlassConfusionMatrix(C).update (or
MulticlassAccuracy(C) with FEWBINS_KIND=acc) on N x C bf16 (FEWBINS_N, default 1 M; FEWBINS_C, default 10), 20 calls."""
import os

import torch

import torchmetrics_amd as tm

C = int(os.environ.get("FEWBINS_C", "10"))
N = int(os.environ.get("FEWBINS_N", str(1 << 20)))
kind = os.environ.get("FEWBINS_KIND", "confmat")
m = (tm.MulticlassAccuracy(C) if kind == "acc" else tm.MulticlassConfusionMatrix(C)).cuda()
g = torch.Generator(device="cuda").manual_seed(0)
p = torch.rand(N, C, device="cuda", generator=g).to(torch.bfloat16)
t = torch.randint(0, C, (N,), device="cuda", generator=g)
for _ in range(20):
    m.update(p, t)
torch.cuda.synchronize()
