import torch, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torchmetrics_amd as tm
from torchmetrics_amd import ops, regression as R
k, n = 1, 1000
def members():
    return {"mse": R.MeanSquaredError(num_outputs=k), "r2": R.R2Score(num_outputs=k), "pearson": R.PearsonCorrCoef(num_outputs=k),
            "concordance": R.ConcordanceCorrCoef(num_outputs=k), "ev": R.ExplainedVariance(), "mae": R.MeanAbsoluteError(),
            "mape": R.MeanAbsolutePercentageError(), "mink": R.MinkowskiDistance(p=3.0), "logcosh": R.LogCoshError(),
            "smape": R.SymmetricMeanAbsolutePercentageError()}
for merged in (True, False):
    gpu = tm.MetricCollection(members(), compute_groups=True).cuda()
    single = {kk: m.cuda() for kk, m in members().items()}
    cpu = members()
    g = torch.Generator().manual_seed(5)
    for step in range(3):
        x = torch.randn(n, generator=g) + 2
        y = x + 0.5 * torch.randn(n, generator=g)
        if merged: gpu.update(x.cuda(), y.cuda())
        for m in cpu.values(): m.update(x, y)
        for m in single.values(): m.update(x.cuda(), y.cuda())
    out = gpu.compute() if merged else {}
    for name, m in cpu.items():
        print(merged, name, float(out[name]) if merged else None, float(single[name].compute()), float(m.compute()))
