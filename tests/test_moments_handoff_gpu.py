"""The multi-block hand-off of the streaming-moments kernel (``csrc/regression/moments.hip`` moments_handoff_kernel,
taken for 8192 <= n * k <= 65536) relies on gfx950's write-through (sc1) stores and sc1 loads instead of the HIP
memory model's release / acquire fences (see the note in the kernel).  These tests pin that assumption to the target:
every returned sum is checked against an fp64 torch reference, many times, with the hand-off blocks racing a
bandwidth-heavy kernel on a second stream (uneven load: the last arriver differs from run to run)."""
import pytest
import torch

from torchmetrics_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_sums(p, t):
    p, t = p.double(), t.double()
    e = p - t
    return {
        ops.SSE: (e * e).sum(0), ops.SAE: e.abs().sum(0), ops.SP: p.sum(0), ops.ST: t.sum(0),
        ops.SPP: (p * p).sum(0), ops.STT: (t * t).sum(0), ops.SPT: (p * t).sum(0),
        ops.COUNT: torch.full((p.shape[1],), float(p.shape[0]), dtype=torch.float64, device=p.device),
    }


@pytest.mark.parametrize("k", [1, 2, 4])
def test_handoff_sums_under_uneven_load(k):
    ids = [ops.SSE, ops.SAE, ops.SP, ops.ST, ops.SPP, ops.STT, ops.SPT, ops.COUNT]
    g = torch.Generator(device=DEV).manual_seed(11 + k)
    side = torch.cuda.Stream()
    noise_a = torch.randn(4096, 4096, device=DEV)
    sizes = [8192 // k, 8192 // k + 3, 20000 // k, 65536 // k, 12345 // k]
    for rep in range(40):
        n = sizes[rep % len(sizes)]
        p = torch.randn(n, k, generator=g, device=DEV)
        t = p * 0.5 + torch.randn(n, k, generator=g, device=DEV)
        with torch.cuda.stream(side):  # a competing kernel: the hand-off's blocks land on busy and idle CUs alike
            noise_a.mul_(1.0000001).add_(1e-7)
        sums = ops.moments_update(p, t, k, ids, [], [], want_sums=True)
        ref = _ref_sums(p, t)
        # per-element products are f32 (sums f64): rtol 1e-6 is far below what one stale or missing partial row of
        # a block (>= 1/128 of the sum) would cost; the count must be exact
        assert torch.equal(sums[:, ops.COUNT], ref[ops.COUNT]), f"rep {rep} n {n}: count"
        for sid, want in ref.items():
            torch.testing.assert_close(sums[:, sid], want, rtol=1e-6, atol=1e-4,
                                       msg=lambda m: f"rep {rep} n {n} sum {sid}: {m}")
    torch.cuda.synchronize()


def test_handoff_metrics_stream_match_fp64():
    """MSE / Pearson / R2 through the hand-off, 30 updates of 8192 pairs, equal the fp64 closed forms."""
    from torchmetrics_amd import regression as R

    g = torch.Generator(device=DEV).manual_seed(5)
    ms = [R.MeanSquaredError().to(DEV), R.PearsonCorrCoef().to(DEV), R.R2Score().to(DEV)]
    ps, ts = [], []
    for _ in range(30):
        p = torch.randn(8192, generator=g, device=DEV)
        t = 0.3 * p + torch.randn(8192, generator=g, device=DEV)
        ps.append(p)
        ts.append(t)
        for m in ms:
            m.update(p, t)
    p, t = torch.cat(ps).double(), torch.cat(ts).double()
    mse = ((p - t) ** 2).mean()
    pc = torch.corrcoef(torch.stack([p, t]))[0, 1]
    r2 = 1 - ((t - p) ** 2).sum() / ((t - t.mean()) ** 2).sum()
    for m, want in zip(ms, (mse, pc, r2)):
        torch.testing.assert_close(m.compute().double(), want, rtol=1e-5, atol=1e-6)
