"""BERTScore / InfoLM with a tiny random-init local BERT (no network, no pretrained weights).  The oracle is a
per-pair plain-loop evaluation of the published formulas on the same model (bert_score package not installed)."""
import math

import pytest
import torch

transformers = pytest.importorskip("transformers")

from torchmetrics_amd.functional.text import bert_score, infolm  # noqa: E402
from torchmetrics_amd.text import BERTScore, InfoLM  # noqa: E402

WORDS = "the cat sat on a mat dog ran far away is there hello world quick brown fox jumps over lazy".split()
PREDS = ["the cat sat on the mat", "hello world", "a quick brown fox jumps over the lazy dog", "dog ran"]
TARGET = ["there is a cat on the mat", "hello there world", "the quick fox jumps", "the dog ran far away"]


@pytest.fixture(scope="module")
def tiny_bert(tmp_path_factory):
    d = tmp_path_factory.mktemp("tinybert")
    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", *WORDS]
    (d / "vocab.txt").write_text("\n".join(vocab) + "\n")
    tok = transformers.BertTokenizer(str(d / "vocab.txt"), do_lower_case=True)
    torch.manual_seed(0)
    cfg = transformers.BertConfig(vocab_size=len(vocab), hidden_size=32, num_hidden_layers=2, num_attention_heads=2,
                                  intermediate_size=64, max_position_embeddings=64)
    model = transformers.BertForMaskedLM(cfg).eval()
    tok.save_pretrained(str(d))
    model.save_pretrained(str(d))
    return str(d), tok, model


def _oracle_bert(model, tok, preds, target, layer=-1, idf=False):
    enc = model.bert if hasattr(model, "bert") else model
    docs = [tok(t)["input_ids"] for t in target]
    n = len(target)
    df = {}
    for d in docs:
        for t in set(d):
            df[t] = df.get(t, 0) + 1
    idf_of = lambda t: math.log((n + 1) / (df.get(t, 0) + 1))  # noqa: E731
    out = []
    for p, t in zip(preds, target):
        emb, w = [], []
        for s in (p, t):
            ids = tok(s, return_tensors="pt")["input_ids"]
            with torch.no_grad():
                h = enc(ids, torch.ones_like(ids), output_hidden_states=True).hidden_states[layer][0]
            h = h / h.norm(dim=-1, keepdim=True)
            h[0] = 0
            h[-1] = 0  # [CLS] / [SEP] embeddings zeroed (they still take part in the max as 0-similarities)
            ww = torch.tensor([idf_of(x) if idf else 1.0 for x in ids[0].tolist()])
            ww[0] = ww[-1] = 0
            emb.append(h)
            w.append(ww / ww.sum())
        cos = emb[0] @ emb[1].T
        prec = (cos.max(1).values * w[0]).sum().item()
        rec = (cos.max(0).values * w[1]).sum().item()
        out.append((prec, rec, 2 * prec * rec / (prec + rec)))
    return torch.tensor(out)


@pytest.mark.parametrize("idf", [False, True])
def test_bert_score_vs_oracle(tiny_bert, idf):
    path, tok, model = tiny_bert
    res = bert_score(PREDS, TARGET, model_name_or_path=path, idf=idf, batch_size=3, num_layers=2)
    ref = _oracle_bert(model, tok, PREDS, TARGET, layer=2, idf=idf)
    got = torch.stack([res["precision"], res["recall"], res["f1"]], 1)
    assert torch.allclose(got, ref, atol=1e-5)


def test_bert_score_module_and_all_layers(tiny_bert):
    path, tok, model = tiny_bert
    m = BERTScore(model_name_or_path=path, num_layers=1, batch_size=2, max_length=32)
    m.update(PREDS[:2], TARGET[:2])
    m.update(PREDS[2:], TARGET[2:])
    out = m.compute()
    ref = _oracle_bert(model, tok, PREDS, TARGET, layer=1)
    assert torch.allclose(out["f1"], ref[:, 2], atol=1e-5)
    allf = bert_score(PREDS, TARGET, model_name_or_path=path, all_layers=True)
    assert allf["f1"].shape == (3, len(PREDS))
    assert torch.allclose(allf["f1"][1], ref[:, 2], atol=1e-5)


def _oracle_infolm(model, tok, preds, target, temperature=0.25, idf=True, measure="kl_divergence"):
    def dists(sents):
        ids_all = [tok(s)["input_ids"] for s in sents]
        n = len(sents)
        df = {}
        for d in ids_all:
            for t in set(d):
                df[t] = df.get(t, 0) + 1
        res = []
        for ids in ids_all:
            acc, den = 0, 0.0
            for pos in range(1, len(ids) - 1):
                x = torch.tensor([ids])
                x[0, pos] = tok.mask_token_id
                with torch.no_grad():
                    logits = model(x, torch.ones_like(x)).logits[0, pos]
                w = math.log((n + 1) / (df[ids[pos]] + 1)) if idf else 1.0
                acc = acc + torch.softmax(logits / temperature, -1) * w
                den += w
            res.append(acc / den)
        return torch.stack(res)

    p, t = dists(preds), dists(target)
    if measure == "kl_divergence":
        return torch.sum(t * torch.log(p / t), -1)
    return torch.norm(t - p, p=1, dim=-1)


@pytest.mark.parametrize(("measure", "idf"), [("kl_divergence", True), ("l1_distance", False)])
def test_infolm_vs_oracle(tiny_bert, measure, idf):
    path, tok, model = tiny_bert
    mean, sent = infolm(PREDS, TARGET, model_name_or_path=path, idf=idf, information_measure=measure, max_length=32,
                        batch_size=3, verbose=False, return_sentence_level_score=True)
    ref = _oracle_infolm(model, tok, PREDS, TARGET, idf=idf, measure=measure)
    assert torch.allclose(sent, ref, atol=1e-4), (sent, ref)
    m = InfoLM(path, idf=idf, information_measure=measure, max_length=32, verbose=False)
    m.update(PREDS[:2], TARGET[:2])
    m.update(PREDS[2:], TARGET[2:])
    assert torch.allclose(m.compute(), ref.mean(), atol=1e-4)


def test_infolm_param_validation():
    from torchmetrics_amd.functional.text.infolm import _InformationMeasure

    with pytest.raises(ValueError):
        _InformationMeasure("alpha_divergence")
    with pytest.raises(ValueError):
        _InformationMeasure("alpha_divergence", alpha=1.0)
    with pytest.raises(ValueError):
        _InformationMeasure("nope")
    im = _InformationMeasure("ab_divergence", alpha=0.5, beta=0.5)
    p = torch.softmax(torch.randn(3, 7), -1)
    assert torch.isfinite(im(p, p.flip(0))).all()
