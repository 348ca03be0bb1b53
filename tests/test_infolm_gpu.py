"""InfoLM kernels (``csrc/text/infolm.hip``): the one-launch information measure vs the reference formulas
(``F/text/infolm.py:60-215``, torch on the CPU, with ``nan_to_num``), the fused softmax / weight / per-sentence sum vs
``softmax`` + ``index_add``, and end-to-end InfoLM on a tiny random BERT on the GPU vs the CPU path."""
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.functional.text.infolm import _InformationMeasure

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

CASES = [("kl_divergence", None, None), ("alpha_divergence", 0.3, None), ("beta_divergence", None, 0.7),
         ("ab_divergence", 0.4, 0.6), ("renyi_divergence", 0.5, None), ("l1_distance", None, None),
         ("l2_distance", None, None), ("l_infinity_distance", None, None), ("fisher_rao_distance", None, None)]


def _dists(n, v, seed, zeros=False):
    g = torch.Generator().manual_seed(seed)
    p = torch.softmax(torch.randn(n, v, generator=g) * 2, -1)
    t = torch.softmax(torch.randn(n, v, generator=g) * 2, -1)
    if zeros:  # exact zeros: KL terms 0 * log(p / 0) are NaN -> the row scores 0 after nan_to_num, as the reference
        t[0, :5] = 0
        p[1, 7] = 0
    return p, t


@pytest.mark.parametrize("measure,alpha,beta", CASES)
@pytest.mark.parametrize("zeros", [False, True])
def test_info_measure_matches_reference(measure, alpha, beta, zeros):
    p, t = _dists(7, 30522, 3, zeros)
    im = _InformationMeasure(measure, alpha, beta)
    got = im(p.to(DEV), t.to(DEV)).cpu()
    # CPU path = the reference's ops, in fp64 for a tight oracle; its nan_to_num maps -inf to the fp64 minimum, which
    # is the fp32 minimum once the fp32 reference's range is applied
    fmax = torch.finfo(torch.float32).max
    ref = im(p.double(), t.double()).clamp(-fmax, fmax).float()
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_accumulate_matches_softmax_index_add(dtype):
    g = torch.Generator().manual_seed(1)
    rows = torch.tensor([0, 0, 0, 2, 2, 3, 5, 5, 5, 5])
    v = 4099
    logits = (torch.randn(rows.numel(), v, generator=g) * 3).to(dtype)
    w = torch.rand(rows.numel(), generator=g)
    acc = torch.full((6, v), 0.5, device=DEV)  # accumulated into, in place
    ops.infolm_accumulate(logits.to(DEV), 0.25, w, rows, acc)
    ref = torch.full((6, v), 0.5).index_add_(0, rows, torch.softmax(logits.float() / 0.25, -1) * w[:, None])
    torch.testing.assert_close(acc.cpu(), ref, rtol=1e-5, atol=1e-7)


def test_infolm_end_to_end_gpu_vs_cpu(tmp_path):
    transformers = pytest.importorskip("transformers")
    from torchmetrics_amd.functional.text import infolm

    words = "the cat sat on a mat dog ran far away is there hello world quick brown fox jumps over lazy".split()
    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", *words]
    (tmp_path / "vocab.txt").write_text("\n".join(vocab) + "\n")
    tok = transformers.BertTokenizer(str(tmp_path / "vocab.txt"), do_lower_case=True)
    torch.manual_seed(0)
    cfg = transformers.BertConfig(vocab_size=len(vocab), hidden_size=32, num_hidden_layers=2, num_attention_heads=2,
                                  intermediate_size=64, max_position_embeddings=64)
    transformers.BertForMaskedLM(cfg).eval().save_pretrained(str(tmp_path))
    tok.save_pretrained(str(tmp_path))
    preds = ["the cat sat on the mat", "hello world", "a quick brown fox jumps over the lazy dog", "dog ran"]
    target = ["there is a cat on the mat", "hello there world", "the quick fox jumps", "the dog ran far away"]
    for measure, alpha, beta in CASES:
        kw = dict(model_name_or_path=str(tmp_path), information_measure=measure, alpha=alpha, beta=beta, max_length=32,
                  batch_size=3, verbose=False, return_sentence_level_score=True)
        _, gpu = infolm(preds, target, device=DEV, **kw)
        _, cpu = infolm(preds, target, device="cpu", **kw)
        torch.testing.assert_close(gpu.cpu(), cpu, rtol=1e-4, atol=1e-5)
