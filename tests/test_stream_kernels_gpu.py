"""Streaming stat-score kernels (``csrc/classification/stat_scores.hip``): the tiled few-bin multiclass kernel
(``mc_fewbins_tile_kernel``) and the vectorised multilabel kernel (``bin_vec_kernel``), each compared with the CPU
(ATen) implementation of the same op contract -- identical integer workspaces and flags -- on shapes that put the
tile / stride boundaries in every position (ragged last tile, rows < one tile, labels not a multiple of the vector
width -> the other kernel), NaN rows, ignore_index, logits vs probabilities, invalid targets."""
import pytest
import torch

from torchmetrics_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _mc(preds, target, C, ignore, mode, dev):
    out = torch.zeros(C * C if mode == ops.MC_CONFMAT else 3 * C + 1, dtype=torch.int64, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.mc_update(preds.to(dev), target.to(dev), out, flag, C, ignore, mode, False)
    return out.cpu(), int(flag.item())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("C", [2, 3, 10, 16, 31])
@pytest.mark.parametrize("N", [1, 255, 2049, 100_003, 1 << 20])
@pytest.mark.parametrize("mode", [0, 1])
def test_fewbins_tiled_matches_cpu(dtype, C, N, mode):
    if mode == ops.MC_CONFMAT and C * C > 256:
        pytest.skip("not a few-bin confusion matrix")
    g = torch.Generator().manual_seed(C * 1000 + N % 997)
    preds = torch.randn(N, C, generator=g).to(dtype)
    target = torch.randint(0, C, (N,), generator=g)
    gg, fg = _mc(preds, target, C, None, mode, DEV)
    cc, fc = _mc(preds, target, C, None, mode, "cpu")
    assert torch.equal(gg, cc)
    assert fg == fc == 0


@pytest.mark.parametrize("ignore", [0, -1])
def test_fewbins_tiled_nan_ties_ignore_and_bad_target(ignore):
    C, N = 10, 70_001
    preds = torch.randn(N, C).to(torch.bfloat16)
    preds[::5] = 0.0  # all-tie rows: first index
    preds[1::13, 3] = float("nan")  # NaN wins
    preds[2::17, 7] = float("inf")
    target = torch.randint(0, C, (N,))
    target[::9] = ignore
    gg, fg = _mc(preds, target, C, ignore, 1, DEV)
    cc, fc = _mc(preds, target, C, ignore, 1, "cpu")
    assert torch.equal(gg, cc) and fg == fc == 0
    bad = target.clone()
    bad[N - 1] = C + 3
    _, fg = _mc(preds, bad, C, ignore, 1, DEV)
    assert fg & 1  # target out of range


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C", [7, 10, 16])
def test_fewbins_ordinal_rows_signed_zero_nan_payloads_inf(dtype, C):
    """The 16-bit rows go through order-preserving ordinals (row_argmax_ord16); every row where ordinals are not exact
    (a max of +-0, negative NaN, NaN payloads, a NaN next to +inf) must still match torch.argmax."""
    N = 50_003
    g = torch.Generator().manual_seed(C)
    preds = torch.randn(N, C, generator=g).to(dtype)
    bits = preds.view(torch.int16)
    preds[0::7] = -preds[0::7].abs()  # all-negative rows
    preds[1::11] = 0.0
    preds[1::11, C - 1] = -0.0  # +0 / -0 ties: first column
    preds[2::11] = -0.0
    preds[2::11, C // 2] = 0.0
    preds[3::11] = -1.0
    preds[3::11, 1] = -0.0  # max is -0 alone
    bits[4::13, C // 3] = -1  # 0xffff: a negative NaN
    bits[5::13, C - 2] = 0x7FC1 if dtype == torch.bfloat16 else 0x7E01  # positive NaN with a payload
    preds[5::13, 0] = float("inf")
    preds[6::17, 1] = float("-inf")
    preds[7::19] = float("inf")  # all +inf: first column
    target = torch.randint(0, C, (N,), generator=g)
    for mode in (0, 1):
        if mode == ops.MC_CONFMAT and C * C > 256:
            continue
        gg, fg = _mc(preds, target, C, None, mode, DEV)
        cc, fc = _mc(preds, target, C, None, mode, "cpu")
        assert torch.equal(gg, cc) and fg == fc == 0


def test_fewbins_tiled_unaligned_input_takes_the_other_kernel():
    C, N = 10, 10_000
    base = torch.randn(N * C + 1).to(torch.bfloat16)
    preds = base[1:].view(N, C)  # 2-byte offset: not 16-byte aligned
    target = torch.randint(0, C, (N,))
    gg, _ = _mc(preds, target, C, None, 1, DEV)
    cc, _ = _mc(preds.contiguous(), target, C, None, 1, "cpu")
    assert torch.equal(gg, cc)


def _bin(preds, target, L, ignore, dev, threshold=0.5):
    ws = torch.zeros(L * 7, dtype=torch.int64, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    not_prob = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.bin_update(preds.to(dev), target.to(dev), ws, flag, not_prob, L, threshold, ignore, False)
    ops.bin_flush(ws)  # the fold of the per-block rows waits for a finalizer otherwise
    return ws.cpu(), int(flag.item()), int(not_prob.item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("tdtype", [torch.int32, torch.int64])
@pytest.mark.parametrize("L", [65, 68, 100, 256, 1000, 1752])
@pytest.mark.parametrize("logits", [False, True])
def test_multilabel_vec_matches_cpu(dtype, tdtype, L, logits):
    N = 3001
    g = torch.Generator().manual_seed(L)
    preds = (torch.randn(N, L, generator=g) * 3 if logits else torch.rand(N, L, generator=g)).to(dtype)
    target = torch.randint(0, 2, (N, L), generator=g).to(tdtype)
    gg = _bin(preds, target, L, None, DEV)
    cc = _bin(preds, target, L, None, "cpu")
    assert torch.equal(gg[0], cc[0]) and gg[1:] == cc[1:]
    assert gg[2] == int(logits)


@pytest.mark.parametrize("ignore", [-1, 1])
def test_multilabel_vec_ignore_and_bad_target(ignore):
    N, L = 4096, 128
    preds = torch.rand(N, L).to(torch.bfloat16)
    target = torch.randint(0, 2, (N, L))
    target[::3, ::5] = ignore
    preds[7, 9] = 1.5  # one non-probability: the logits reading for the whole call
    gg = _bin(preds, target, L, ignore, DEV)
    cc = _bin(preds, target, L, ignore, "cpu")
    assert torch.equal(gg[0], cc[0]) and gg[1:] == cc[1:]
    bad = target.clone()
    bad[N - 1, L - 1] = 2
    _, flag, _ = _bin(preds, bad, L, ignore, DEV)
    assert flag & 4  # target not binary


def test_multilabel_module_values_on_vec_path():
    import torchmetrics_amd as tm

    N, L = 16384, 1000
    p = torch.rand(N, L).to(torch.bfloat16)
    t = torch.randint(0, 2, (N, L), dtype=torch.int32)
    m = tm.MultilabelF1Score(L).to(DEV)
    m.update(p.to(DEV), t.to(DEV))
    ref = tm.MultilabelF1Score(L)
    ref.update(p, t)
    torch.testing.assert_close(m.compute().cpu(), ref.compute())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("odd", ["none", "neg_zero", "one", "above_one", "tiny_negative", "nan", "neg_nan", "inf"])
def test_multilabel_vec_probability_range_edges(dtype, odd):
    """bin_vec_kernel decides "all scores in [0, 1]" from a packed ordinal min / max (OrdRange): -0.0 and 1.0 are in
    range; anything above 1, below -0.0, NaN of either sign or inf is not -- the same reading as the CPU path."""
    N, L = 2048, 128
    g = torch.Generator().manual_seed(17)
    preds = torch.rand(N, L, generator=g).to(dtype)
    target = torch.randint(0, 2, (N, L), generator=g)
    val = {"none": None, "neg_zero": -0.0, "one": 1.0, "above_one": 1.0078125, "tiny_negative": -1e-3,
           "nan": float("nan"), "neg_nan": -float("nan"), "inf": float("inf")}[odd]
    if val is not None:
        preds[N // 2, L // 3] = val
        if odd == "neg_nan":
            bits = preds.view(torch.int16 if dtype != torch.float32 else torch.int32)
            bits[N // 2, L // 3] |= (-32768 if dtype != torch.float32 else -(2 ** 31))
    gg = _bin(preds, target, L, None, DEV)
    cc = _bin(preds, target, L, None, "cpu")
    assert gg[2] == cc[2]  # the probabilities / logits decision
    if odd not in ("nan", "neg_nan"):
        assert torch.equal(gg[0], cc[0])


@pytest.mark.parametrize("dtype,C", [(torch.bfloat16, 2), (torch.bfloat16, 10), (torch.float16, 17),
                                     (torch.bfloat16, 64), (torch.float32, 10), (torch.float32, 31)])
@pytest.mark.parametrize("N", [1, 255, 3000, 100_003, 1 << 22])
def test_fewbins_group_handoff_states(dtype, C, N):
    """Few-class multiclass stats straight into the tp / fp / tn / fn states in one launch (mc_stats_direct ->
    mc_fewbins_tile_kernel's group hand-off: the last block of each group sums its partial rows and adds them to the
    states; tickets re-armed by the kernel): repeated updates of different batches, then the confusion matrix (same
    hand-off, matrix destination), equal to the CPU module."""
    import torchmetrics_amd as tm

    g = torch.Generator().manual_seed(C * 7 + N % 1013)
    ms = tm.MulticlassStatScores(C, average="none").to(DEV)
    cm = tm.MulticlassConfusionMatrix(C).to(DEV)
    rs, rc = tm.MulticlassStatScores(C, average="none"), tm.MulticlassConfusionMatrix(C)
    for i in range(3):
        p = torch.randn(N, C, generator=g).to(dtype)
        t = torch.randint(0, C, (N,), generator=g)
        if i == 1:
            p[::3] = 0.0  # ties: first index
        ms.update(p.to(DEV), t.to(DEV))
        cm.update(p.to(DEV), t.to(DEV))
        rs.update(p.float(), t)
        rc.update(p.float(), t)
    for k in ("tp", "fp", "tn", "fn"):
        assert torch.equal(getattr(ms, k).cpu(), getattr(rs, k)), k
    assert torch.equal(ms.compute().cpu(), rs.compute())
    assert torch.equal(cm.compute().cpu(), rc.compute())
