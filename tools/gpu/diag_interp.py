"""Diagnostic: where does the fp64 device interp_mean differ from the torch op chain (tests/test_macro_curves.py)?"""
import torch

from torchmetrics_amd import ops


def ref_interp(x, xp, fp):
    den = xp[1:] - xp[:-1]
    den[den == 0.0] = 1
    m = (fp[1:] - fp[:-1]) / den
    b = fp[:-1] - (m * xp[:-1])
    idx = torch.searchsorted(xp.contiguous(), x.contiguous(), right=True) - 1
    idx = torch.clamp(idx, 0, len(m) - 1)
    return m[idx] * x + b[idx], idx


def main() -> None:
    dtype = torch.float64
    g = torch.Generator().manual_seed(3)
    xs = [torch.rand(n, generator=g, dtype=dtype) for n in (2, 7, 50, 3)]
    xs[1] = xs[1].sort().values
    ys = [torch.rand(x.numel(), generator=g, dtype=dtype) for x in xs]
    xs[2][10] = xs[2][11]
    grid = torch.cat([torch.cat(xs), torch.tensor([-1.0, 2.0], dtype=dtype)]).sort().values
    off = torch.tensor([0, 2, 9, 59, 62])
    out = ops.interp_mean(grid.cuda(), torch.cat(xs).cuda(), torch.cat(ys).cuda(), off.cuda()).cpu()
    cpu = ops.interp_mean(grid, torch.cat(xs), torch.cat(ys), off)
    ref = torch.zeros_like(grid)
    for x, y in zip(xs, ys):
        ref += ref_interp(grid, x, y)[0]
    ref = ref / 4
    bad = (out != ref).nonzero().flatten().tolist()
    print("mismatches dev-vs-ref", len(bad), "cpu-vs-ref", int((cpu != ref).sum()), "dev-vs-cpu", int((out != cpu).sum()))
    for j in bad[:8]:
        print(j, float(grid[j]).hex(), float(out[j]).hex(), float(ref[j]).hex(), float(cpu[j]).hex())
        for c, (x, y) in enumerate(zip(xs, ys)):
            v, idx = ref_interp(grid[j : j + 1], x, y)
            one = ops.interp_mean(grid[j : j + 1].cuda(), x.cuda(), y.cuda(), torch.tensor([0, x.numel()]).cuda())
            print("   class", c, "idx", int(idx), float(v).hex(), float(one.cpu()).hex())


if __name__ == "__main__":
    main()
