"""Text metrics (reference ``tests/unittests/text``).  jiwer / sacrebleu / nltk / rouge_score are not installed, so
parity is pinned against (a) the reference's own docstring values and hard-coded fixtures (nltk distance cases,
RWTH EED numbers) and (b) plain-Python oracles of the textbook algorithms written here."""
import random
from collections import Counter
from math import exp, log

import numpy as np
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd import functional as F
from torchmetrics_amd.functional.text import eed as eed_mod
from torchmetrics_amd.text import (
    BLEUScore,
    CharErrorRate,
    CHRFScore,
    EditDistance,
    ExtendedEditDistance,
    MatchErrorRate,
    Perplexity,
    ROUGEScore,
    SacreBLEUScore,
    SQuAD,
    TranslationEditRate,
    WordErrorRate,
    WordInfoLost,
    WordInfoPreserved,
)

PREDS = ["this is the prediction", "there is an other sample"]
TARGET = ["this is the reference", "there is another one"]
HYP_A = "It is a guide to action which ensures that the military always obeys the commands of the party"
REF_1A = "It is a guide to action that ensures that the military will forever heed Party commands"
REF_2A = "It is a guiding principle which makes the military forces always being under the command of the Party"
HYP_B = "he read the book because he was interested in world history"
REF_1B = "he was interested in world history because he read the book"
REF_2B = "It is the practical guide for the army always to heed the directions of the party"
HYP_C = "the cat the   cat on the mat "
REF_1C = "the  cat is     on the mat "
REF_2C = "there is a   cat on the mat"


def _lev(a, b, sub=1):
    prev = list(range(len(b) + 1))
    for i in range(1, len(a) + 1):
        cur = [i] + [0] * len(b)
        for j in range(1, len(b) + 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (0 if a[i - 1] == b[j - 1] else sub))
        prev = cur
    return prev[-1]


def _random_sentences(n, seed, words="a bb ccc the cat sat on mat dog ran far away".split()):
    rng = random.Random(seed)
    return [" ".join(rng.choices(words, k=rng.randint(0, 14))) for _ in range(n)]


# --------------------------------------------------------------------------------------------- edit distances
NLTK_CASES = [
    ("abc", "ca", 1, 3), ("abc", "ca", 5, 3), ("wants", "wasp", 1, 3), ("wants", "wasp", 5, 3),
    ("rain", "shine", 1, 3), ("rain", "shine", 2, 5), ("acbdef", "abcdef", 1, 2), ("acbdef", "abcdef", 2, 2),
    ("lnaguaeg", "language", 1, 4), ("lnaguaeg", "language", 2, 4), ("lnaugage", "language", 1, 3),
    ("lnaugage", "language", 2, 4), ("lngauage", "language", 1, 2), ("lngauage", "language", 2, 2),
    ("wants", "swim", 1, 5), ("wants", "swim", 2, 7), ("kitten", "sitting", 1, 3), ("kitten", "sitting", 2, 5),
    ("duplicated", "duuplicated", 1, 1), ("duplicated", "duuplicated", 2, 1),
    ("very duplicated", "very duuplicateed", 2, 2),
]


@pytest.mark.parametrize(("left", "right", "cost", "expected"), NLTK_CASES)
def test_edit_distance_fixtures(left, right, cost, expected):
    assert F.edit_distance([left], [right], substitution_cost=cost).item() == expected


def _pack(seqs):
    off = np.zeros(len(seqs) + 1, dtype=np.int64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    ids = np.concatenate([np.asarray(s, dtype=np.int32) for s in seqs]) if off[-1] else np.zeros(0, np.int32)
    return torch.from_numpy(ids), torch.from_numpy(off)


def _lev_cases(seed=0, n=60):
    rng = np.random.default_rng(seed)
    ps, rs = [], []
    for k in range(n):
        lp, lr = int(rng.integers(0, 140)), int(rng.integers(0, 140))
        if k % 7 == 0:
            lp = 0
        ps.append(rng.integers(0, 5, lp))
        rs.append(rng.integers(0, 5, lr))
    return ps, rs


@pytest.mark.parametrize("beam", [False, True])
@pytest.mark.parametrize("sub", [1, 2])
def test_levenshtein_native_vs_python(beam, sub):
    """Native host DP (when built) == Python DP, with and without the tercom beam."""
    ps, rs = _lev_cases()
    p, po = _pack(ps)
    r, ro = _pack(rs)
    ref = torch.empty(len(ps), dtype=torch.int64)
    from torchmetrics_amd.ops import _cpu

    _cpu.levenshtein(p, po, r, ro, ref, 1, 1, sub, beam, 0)
    if not beam:
        assert ref.tolist() == [_lev(a.tolist(), b.tolist(), sub) for a, b in zip(ps, rs)]
    got = ops.levenshtein(p, po, r, ro, 1, 1, sub, beam)
    assert torch.equal(got, ref)


def test_error_rate_docstrings():
    assert torch.isclose(F.word_error_rate(PREDS, TARGET), torch.tensor(0.5))
    assert torch.isclose(F.char_error_rate(PREDS, TARGET), torch.tensor(0.3415), atol=1e-4)
    assert torch.isclose(F.match_error_rate(PREDS, TARGET), torch.tensor(0.4444), atol=1e-4)
    assert torch.isclose(F.word_information_lost(PREDS, TARGET), torch.tensor(0.6528), atol=1e-4)
    assert torch.isclose(F.word_information_preserved(PREDS, TARGET), torch.tensor(0.3472), atol=1e-4)


def _rates_oracle(preds, target):
    err = tot = mx = pt = tt = cerr = ctot = 0
    for p, t in zip(preds, target):
        pw, tw = p.split(), t.split()
        e = _lev(pw, tw)
        err += e
        tot += len(tw)
        mx += max(len(pw), len(tw))
        pt += len(pw)
        tt += len(tw)
        cerr += _lev(list(p), list(t))
        ctot += len(t)
    hits = err - mx
    wip = (hits / tt) * (hits / pt)
    return {"wer": err / tot, "cer": cerr / ctot, "mer": err / mx, "wip": wip, "wil": 1 - wip}


@pytest.mark.parametrize(
    ("cls", "key"),
    [(WordErrorRate, "wer"), (CharErrorRate, "cer"), (MatchErrorRate, "mer"), (WordInfoLost, "wil"),
     (WordInfoPreserved, "wip")],
)
def test_error_rate_modules(cls, key, device="cpu"):
    batches = [(_random_sentences(8, s), _random_sentences(8, s + 100)) for s in range(4)]
    for b in batches:  # guarantee non-empty references
        b[1][0] = "the cat"
        b[0][0] = "a dog"
    m = cls().to(device)
    for p, t in batches:
        m.update(p, t)
    allp = [x for p, _ in batches for x in p]
    allt = [x for _, t in batches for x in t]
    assert np.isclose(m.compute().item(), _rates_oracle(allp, allt)[key], atol=1e-5)


def test_edit_distance_module_reductions():
    p, t = ["rain", "kitten", "abc"], ["shine", "sitting", "ca"]
    for red, exp_val in (("mean", 3.0), ("sum", 9), ("none", [3, 3, 3])):
        m = EditDistance(reduction=red)
        m.update(p[:2], t[:2])
        m.update(p[2:], t[2:])
        out = m.compute()
        assert out.tolist() == exp_val if red == "none" else np.isclose(out.item(), exp_val)
    assert F.edit_distance([], []) == 0
    with pytest.raises(ValueError):
        EditDistance(substitution_cost=-1)


# ------------------------------------------------------------------------------------------------- BLEU family
def _bleu_oracle(preds, targets, n_gram=4, smooth=False):
    num, den = [0] * n_gram, [0] * n_gram
    plen = tlen = 0
    for p, ts in zip(preds, targets):
        pw = p.split()
        tws = [t.split() for t in ts]
        plen += len(pw)
        diffs = [abs(len(pw) - len(t)) for t in tws]
        tlen += len(tws[diffs.index(min(diffs))])
        for n in range(1, n_gram + 1):
            pc = Counter(tuple(pw[i:i + n]) for i in range(len(pw) - n + 1))
            rc = Counter()
            for t in tws:
                rc |= Counter(tuple(t[i:i + n]) for i in range(len(t) - n + 1))
            num[n - 1] += sum((pc & rc).values())
            den[n - 1] += sum(pc.values())
    if min(num) == 0:
        return 0.0
    prec = [(num[i] + 1) / (den[i] + 1) if smooth and i > 0 else num[i] / den[i] for i in range(n_gram)]
    geo = exp(sum(log(x) / n_gram for x in prec))
    bp = 1.0 if plen > tlen else exp(1 - tlen / plen)
    return bp * geo


def test_bleu_docstring_and_oracle():
    assert torch.isclose(F.bleu_score(["the cat is on the mat"], [["there is a cat on the mat", "a cat is on the mat"]]),
                         torch.tensor(0.7598), atol=1e-4)
    preds = [HYP_A, HYP_B, HYP_C]
    tgts = [[REF_1A, REF_2A], [REF_1B, REF_2B], [REF_1C, REF_2C]]
    for n in (1, 2, 3, 4):
        for smooth in (False, True):
            assert np.isclose(F.bleu_score(preds, tgts, n_gram=n, smooth=smooth).item(),
                              _bleu_oracle(preds, tgts, n, smooth), atol=1e-6)
    m = BLEUScore(smooth=True)
    m.update(preds[:2], tgts[:2])
    m.update(preds[2:], tgts[2:])
    assert np.isclose(m.compute().item(), _bleu_oracle(preds, tgts, 4, True), atol=1e-6)


def test_sacrebleu():
    sb = SacreBLEUScore()
    assert torch.isclose(sb(["the cat is on the mat"], [["there is a cat on the mat", "a cat is on the mat"]]),
                         torch.tensor(0.7598), atol=1e-4)
    # 13a splits punctuation, so a trailing period is an extra token on both sides
    v = F.sacre_bleu_score(["the cat is on the mat."], [["a cat is on the mat."]], tokenize="13a")
    assert np.isclose(v.item(), _bleu_oracle(["the cat is on the mat ."], [["a cat is on the mat ."]]), atol=1e-6)
    for tok in ("none", "char", "zh", "intl"):
        assert 0 <= F.sacre_bleu_score(["the cat is on the mat."], [["a cat is on the mat."]], tokenize=tok) <= 1
    with pytest.raises(ValueError):
        SacreBLEUScore(tokenize="nope")


def test_chrf():
    preds, tgt = ["the cat is on the mat"], [["there is a cat on the mat", "a cat is on the mat"]]
    assert torch.isclose(F.chrf_score(preds, tgt), torch.tensor(0.8640), atol=1e-4)
    m = CHRFScore(return_sentence_level_score=True)
    m.update([HYP_A, HYP_B], [[REF_1A, REF_2A], [REF_1B, REF_2B]])
    m.update([HYP_C], [[REF_1C, REF_2C]])
    score, sent = m.compute()
    ref_score, ref_sent = F.chrf_score([HYP_A, HYP_B, HYP_C], [[REF_1A, REF_2A], [REF_1B, REF_2B], [REF_1C, REF_2C]],
                                       return_sentence_level_score=True)
    assert torch.isclose(score, ref_score) and torch.allclose(sent, ref_sent)
    assert "total_preds_char_6_grams" in m.state_dict() or hasattr(m, "total_preds_char_6_grams")


def test_ter_and_eed():
    assert torch.isclose(F.translation_edit_rate(["the cat is on the mat"],
                                                 [["there is a cat on the mat", "a cat is on the mat"]]),
                         torch.tensor(0.1538), atol=1e-4)
    ter = TranslationEditRate(return_sentence_level_score=True)
    ter.update([HYP_A], [[REF_1A, REF_2A]])
    ter.update([HYP_B], [[REF_1B, REF_2B]])
    val, sent = ter.compute()
    assert val.item() > 0 and sent.numel() == 2
    assert F.translation_edit_rate(["a b c"], [["a b c"]]) == 0
    # RWTH reference numbers pinned in the reference's test-suite (T/text/test_eed.py:33-34)
    ans_1, ans_2 = 0.24248056001808083, 0.19152276295133436
    for native in (True, False):
        orig = eed_mod.ops.native_available
        if not native:
            eed_mod.ops.native_available = lambda: False
        try:
            v1 = F.extended_edit_distance([HYP_A, HYP_B], [[REF_1A], [REF_1B]])
            v2 = F.extended_edit_distance([HYP_B, HYP_C], [[REF_1B], [REF_1C]])
        finally:
            eed_mod.ops.native_available = orig
        assert np.isclose(v1.item(), ans_1, atol=1e-6) and np.isclose(v2.item(), ans_2, atol=1e-6)
    m = ExtendedEditDistance()
    m.update([HYP_A, HYP_B], [[REF_1A], [REF_1B]])
    m.update([HYP_B, HYP_C], [[REF_1B], [REF_1C]])
    assert np.isclose(m.compute().item(), (ans_1 + ans_2) / 2, atol=1e-6)


def _lcs(a, b):
    t = [[0] * (len(b) + 1) for _ in range(len(a) + 1)]
    for i in range(1, len(a) + 1):
        for j in range(1, len(b) + 1):
            t[i][j] = t[i - 1][j - 1] + 1 if a[i - 1] == b[j - 1] else max(t[i - 1][j], t[i][j - 1])
    return t[-1][-1]


def test_rouge():
    out = F.rouge_score("My name is John", "Is your name John")
    assert np.isclose(out["rouge1_fmeasure"], 0.75) and np.isclose(out["rougeL_fmeasure"], 0.5)
    assert out["rouge2_fmeasure"] == 0
    preds = _random_sentences(12, 5)
    tgts = _random_sentences(12, 6)
    out = F.rouge_score(preds, tgts, rouge_keys=("rougeL",))
    fs = []
    for p, t in zip(preds, tgts):
        pw, tw = p.split(), t.split()
        if not pw or not tw:
            fs.append(0.0)
            continue
        lcs = _lcs(pw, tw)
        pr, rc = lcs / len(pw), lcs / len(tw)
        fs.append(0.0 if pr == rc == 0 else 2 * pr * rc / (pr + rc))
    assert np.isclose(out["rougeL_fmeasure"].item(), np.mean(fs), atol=1e-6)
    m = ROUGEScore(rouge_keys=("rouge1", "rougeL"), accumulate="avg")
    m.update(preds[:6], [[t, p] for t, p in zip(tgts[:6], preds[:6])])
    m.update(preds[6:], [[t, p] for t, p in zip(tgts[6:], preds[6:])])
    res = m.compute()
    assert set(res) == {f"rouge{k}_{t}" for k in ("1", "L") for t in ("fmeasure", "precision", "recall")}


def test_squad():
    preds = [{"prediction_text": "1976", "id": "id1"}, {"prediction_text": "Hello", "id": "id2"}]
    tgt = [{"answers": {"answer_start": [97], "text": ["1976"]}, "id": "id1"},
           {"answers": {"answer_start": [97], "text": ["World"]}, "id": "id2"}]
    out = F.squad(preds, tgt)
    assert out["exact_match"].item() == 50.0 and out["f1"].item() == 50.0
    m = SQuAD()
    m.update(preds[0], tgt[0])
    assert m.compute()["f1"].item() == 100.0
    with pytest.raises(KeyError):
        F.squad({"id": "x"}, tgt)


def _ppl_ref(preds, target, ignore_index=None):
    lp = torch.log_softmax(preds.double().reshape(-1, preds.shape[-1]), 1)
    t = target.reshape(-1)
    mask = torch.ones_like(t, dtype=torch.bool) if ignore_index is None else t != ignore_index
    tt = torch.where(mask, t, torch.zeros_like(t))
    nll = -lp.gather(1, tt[:, None])[:, 0][mask]
    return torch.exp(nll.mean())


def test_perplexity():
    gen = torch.manual_seed(42)
    preds = torch.rand(2, 8, 5, generator=gen)
    target = torch.randint(5, (2, 8), generator=gen)
    target[0, 6:] = -100
    assert torch.isclose(F.perplexity(preds, target, ignore_index=-100), torch.tensor(5.8540), atol=1e-4)
    m = Perplexity(ignore_index=-100)
    m.update(preds[:1], target[:1])
    m.update(preds[1:], target[1:])
    assert torch.isclose(m.compute(), torch.tensor(5.8540), atol=1e-4)
    with pytest.raises(ValueError):
        F.perplexity(preds[0], target)
    with pytest.raises(TypeError):
        F.perplexity(preds, target.int())


# --------------------------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("beam", [False, True])
@pytest.mark.parametrize("sub", [1, 2])
def test_levenshtein_kernel_gpu(beam, sub):
    ps, rs = _lev_cases(seed=3, n=300)
    ps.append(np.random.default_rng(1).integers(0, 30, 3000))  # long row: many 64-column chunks, many beam rows
    rs.append(np.random.default_rng(2).integers(0, 30, 2500))
    p, po = _pack(ps)
    r, ro = _pack(rs)
    ref = torch.empty(len(ps), dtype=torch.int64)
    from torchmetrics_amd.ops import _cpu

    _cpu.levenshtein(p, po, r, ro, ref, 1, 1, sub, beam, 0)
    got = ops.levenshtein(p.cuda(), po.cuda(), r.cuda(), ro.cuda(), 1, 1, sub, beam, int((ro[1:] - ro[:-1]).max()))
    assert torch.equal(got.cpu(), ref)


@pytest.mark.gpu
def test_text_modules_gpu():
    for cls, key in ((WordErrorRate, "wer"), (CharErrorRate, "cer"), (WordInfoLost, "wil")):
        test_error_rate_modules(cls, key, device="cuda")
    m = EditDistance(reduction="sum").cuda()
    m.update(["rain", "kitten"], ["shine", "sitting"])
    assert m.compute().item() == 6 and m.edit_scores.is_cuda


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
@pytest.mark.parametrize("vocab", [5, 37, 32000])
def test_perplexity_kernel_gpu(dtype, vocab):
    g = torch.Generator().manual_seed(vocab)
    preds = (torch.randn(3, 17, vocab, generator=g) * 3).to(dtype)
    target = torch.randint(vocab, (3, 17), generator=g)
    target[0, 5:] = -100
    ref = _ppl_ref(preds, target, -100)
    m = Perplexity(ignore_index=-100).cuda()
    m.update(preds.cuda(), target.cuda())
    tol = 1e-5 if dtype in (torch.float32, torch.float64) else 1e-3
    assert torch.isclose(m.compute().cpu().double(), ref, rtol=tol)
    # gradient through the fused kernel matches autograd of log_softmax
    x = preds.cuda().float().requires_grad_(True)
    F.perplexity(x, target.cuda(), ignore_index=-100).backward()
    x2 = preds.float().clone().requires_grad_(True)
    _ppl_ref(x2, target, -100).float().backward()
    assert torch.allclose(x.grad.cpu(), x2.grad, atol=1e-5)
    bad = Perplexity().cuda()
    bad.update(preds.cuda(), torch.full((3, 17), vocab + 3, device="cuda"))
    with pytest.raises((RuntimeError, ValueError, IndexError)):
        bad.compute()
