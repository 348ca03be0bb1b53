"""One few-class case for counter collection: MulticlassConfusionMatrix(10).update on 1 M x 10 bf16, 20 calls."""
import torch

import torchmetrics_amd as tm

m = tm.MulticlassConfusionMatrix(10).cuda()
g = torch.Generator(device="cuda").manual_seed(0)
p = torch.rand(1 << 20, 10, device="cuda", generator=g).to(torch.bfloat16)
t = torch.randint(0, 10, (1 << 20,), device="cuda", generator=g)
for _ in range(20):
    m.update(p, t)
torch.cuda.synchronize()
