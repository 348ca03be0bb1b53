"""InfoLM (reference ``F/text/infolm.py``).

Each sentence is summarised by the (idf-weighted) average over its non-special tokens of the masked-LM distribution
at that position (token masked, temperature-scaled softmax); the score is an information measure between the
prediction and reference summaries.

MI355X-first scheduling: instead of the reference's one encoder forward per sequence *position* for every batch
(``seq_len`` launches of a ``[B, S]`` batch, ``F/text/infolm.py:300-312``), every (sentence, real-token position)
pair becomes one row of a ``[rows, S]`` masked-input batch, processed in chunks sized to a token budget, and only
the logits at the masked position are gathered -- padding / special positions (weight 0 in the reference) are never
run through the model.
"""
import os
from enum import Enum
from typing import Dict, List, Literal, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.functional.text._embedding import idf_table, idf_weights, progress, sorted_batches

_ALLOWED_INFORMATION_MEASURE_LITERAL = Literal[
    "kl_divergence", "alpha_divergence", "beta_divergence", "ab_divergence", "renyi_divergence", "l1_distance",
    "l2_distance", "l_infinity_distance", "fisher_rao_distance",
]
_MEASURES = ("kl_divergence", "alpha_divergence", "beta_divergence", "ab_divergence", "renyi_divergence",
             "l1_distance", "l2_distance", "l_infinity_distance", "fisher_rao_distance")
_TOKEN_BUDGET = 1 << 16  # rows x seq_len per encoder chunk


class _InformationMeasure:
    """Information measure between discrete distributions (``F/text/infolm.py:60``), with the same parameter checks."""

    def __init__(self, information_measure: str, alpha: Optional[float] = None, beta: Optional[float] = None) -> None:
        im = str(information_measure).lower()
        if im not in _MEASURES:
            raise ValueError(f"Invalid Information measure: `{information_measure}`. Expected one of {_MEASURES}")
        self.information_measure = im
        if im in ("alpha_divergence", "ab_divergence", "renyi_divergence") and not isinstance(alpha, float):
            raise ValueError(f"Parameter `alpha` is expected to be defined for {information_measure}.")
        if im in ("beta_divergence", "ab_divergence") and not isinstance(beta, float):
            raise ValueError(f"Parameter `beta` is expected to be defined for {information_measure}.")
        if im == "alpha_divergence" and alpha in (0, 1):
            raise ValueError(
                f"Parameter `alpha` is expected to be float differened from 0 and 1 for {information_measure}.")
        if im == "beta_divergence" and beta in (0, -1):
            raise ValueError(
                f"Parameter `beta` is expected to be float differened from 0 and -1 for {information_measure}.")
        if im == "ab_divergence" and 0 in (alpha, beta, (alpha or 0) + (beta or 0)):
            raise ValueError(
                "Parameters `alpha`, `beta` and their sum are expected to be differened from 0 for "
                f"{information_measure}.")
        if im == "renyi_divergence" and alpha == 1:
            raise ValueError(f"Parameter `alpha` is expected to be float differened from 1 for {information_measure}.")
        self.alpha = alpha or 0
        self.beta = beta or 0

    def __call__(self, p: Tensor, t: Tensor) -> Tensor:
        fused = ops.info_measure(p, t, self.information_measure, self.alpha, self.beta)  # ROCm: one launch
        if fused is not None:
            return fused
        return torch.nan_to_num(getattr(self, f"_{self.information_measure}")(p, t))

    @staticmethod
    def _kl_divergence(p: Tensor, t: Tensor) -> Tensor:
        return torch.sum(t * torch.log(p / t), dim=-1)

    def _alpha_divergence(self, p: Tensor, t: Tensor) -> Tensor:
        a = self.alpha
        return (1 - torch.sum(t**a * p ** (1 - a), dim=-1)) / (a * (a - 1))

    def _ab_divergence(self, p: Tensor, t: Tensor, alpha: Optional[float] = None) -> Tensor:
        a = self.alpha if alpha is None else alpha
        b = self.beta
        x = torch.log(torch.sum(t ** (b + a), dim=-1)) / (b * (b + a))
        y = torch.log(torch.sum(p ** (b + a), dim=-1)) / (a * (b + a))
        z = torch.log(torch.sum(t**a * p**b, dim=-1)) / (a * b)
        return x + y - z

    def _beta_divergence(self, p: Tensor, t: Tensor) -> Tensor:
        return self._ab_divergence(p, t, alpha=1.0)

    def _renyi_divergence(self, p: Tensor, t: Tensor) -> Tensor:
        a = self.alpha
        return torch.log(torch.sum(t**a * p ** (1 - a), dim=-1)) / (a - 1)

    @staticmethod
    def _l1_distance(p: Tensor, t: Tensor) -> Tensor:
        return torch.norm(t - p, p=1, dim=-1)

    @staticmethod
    def _l2_distance(p: Tensor, t: Tensor) -> Tensor:
        return torch.norm(t - p, p=2, dim=-1)

    @staticmethod
    def _l_infinity_distance(p: Tensor, t: Tensor) -> Tensor:
        return torch.norm(t - p, p=float("inf"), dim=-1)

    @staticmethod
    def _fisher_rao_distance(p: Tensor, t: Tensor) -> Tensor:
        return 2 * torch.acos(torch.clamp(torch.sqrt(p * t).sum(-1), 0, 1))


def _get_special_tokens_map(tokenizer) -> Dict[str, int]:
    return {"mask_token_id": tokenizer.mask_token_id, "pad_token_id": tokenizer.pad_token_id,
            "sep_token_id": tokenizer.sep_token_id, "cls_token_id": tokenizer.cls_token_id}


def _get_token_mask(input_ids: Tensor, pad_token_id: int, sep_token_id: int, cls_token_id: int) -> Tensor:
    return ~(input_ids.eq(pad_token_id) | input_ids.eq(sep_token_id) | input_ids.eq(cls_token_id))


@torch.no_grad()
def _sentence_distributions(model, input_ids: Tensor, attention_mask: Tensor, temperature: float,
                            weights: Optional[Tensor], special: Dict[str, int], batch_size: int,
                            verbose: bool) -> Tensor:
    """``[N, V]`` weighted mean masked-LM distribution per sentence (original row order)."""
    dev = next(model.parameters()).device
    token_mask = _get_token_mask(input_ids, special["pad_token_id"], special["sep_token_id"], special["cls_token_id"])
    out: Optional[Tensor] = None
    for rows, ln in progress(list(sorted_batches(attention_mask, batch_size)), verbose):
        ids = input_ids[rows, :ln]
        am = attention_mask[rows, :ln]
        tm = token_mask[rows, :ln]
        w = tm.float() if weights is None else weights[rows, :ln] * tm
        r_idx, pos = torch.nonzero(tm, as_tuple=True)  # only real tokens contribute (row-major: sorted by row)
        acc = None
        chunk = max(1, _TOKEN_BUDGET // ln)
        for s in range(0, r_idx.numel(), chunk):
            ri, pi = r_idx[s:s + chunk], pos[s:s + chunk]
            masked = ids[ri].clone()
            masked[torch.arange(ri.numel()), pi] = special["mask_token_id"]
            logits = model(masked.to(dev), am[ri].to(dev)).logits
            logits = logits[torch.arange(ri.numel(), device=dev), pi.to(dev)]
            if logits.is_cuda:
                # softmax, weight and per-sentence sum in two launches, accumulated in place (ops.infolm_accumulate)
                if acc is None:
                    acc = torch.zeros(ids.shape[0], logits.shape[-1], device=dev)
                ops.infolm_accumulate(logits, temperature, w[ri, pi], ri.cpu(), acc)
                continue
            prob = torch.softmax(logits.float() / temperature, dim=-1) * w[ri, pi].to(dev)[:, None]
            part = torch.zeros(ids.shape[0], prob.shape[-1], device=dev).index_add_(0, ri.to(dev), prob)
            acc = part if acc is None else acc + part
        denom = w.sum(1).to(dev)[:, None]
        if acc is None:
            acc = torch.zeros(ids.shape[0], model.config.vocab_size, device=dev)
        dist = acc / denom
        if out is None:
            out = torch.empty(input_ids.shape[0], dist.shape[-1], device=dev)
        out[rows.to(dev)] = dist
    return out if out is not None else torch.zeros(0)


def _load_tokenizer_and_model(model_name_or_path: Union[str, os.PathLike],
                              device: Optional[Union[str, torch.device]] = None):
    from transformers import AutoModelForMaskedLM, AutoTokenizer

    tokenizer = AutoTokenizer.from_pretrained(model_name_or_path)
    model = AutoModelForMaskedLM.from_pretrained(model_name_or_path)
    model.eval()
    model.to(device)
    return tokenizer, model


def _infolm_update(preds: Union[str, Sequence[str]], target: Union[str, Sequence[str]], tokenizer,
                   max_length: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    if not isinstance(preds, (str, list)):
        preds = list(preds)
    if not isinstance(target, (str, list)):
        target = list(target)
    p = tokenizer(preds, padding="max_length", max_length=max_length, truncation=True, return_tensors="pt")
    t = tokenizer(target, padding="max_length", max_length=max_length, truncation=True, return_tensors="pt")
    return p.input_ids, p.attention_mask, t.input_ids, t.attention_mask


def _infolm_compute(model, preds_input_ids: Tensor, preds_attention_mask: Tensor, target_input_ids: Tensor,
                    target_attention_mask: Tensor, temperature: float, idf: bool,
                    information_measure_cls: _InformationMeasure, special_tokens_map: Dict[str, int],
                    batch_size: int = 64, verbose: bool = True) -> Tensor:
    """Sentence-level InfoLM scores ``[N]``.  IDF tables are computed per side (as the reference's datasets do)."""
    pw = tw = None
    if idf:
        pt, pd = idf_table(preds_input_ids)
        tt, td = idf_table(target_input_ids)
        pw, tw = idf_weights(preds_input_ids, pt, pd), idf_weights(target_input_ids, tt, td)
    p = _sentence_distributions(model, preds_input_ids, preds_attention_mask, temperature, pw, special_tokens_map,
                                batch_size, verbose)
    t = _sentence_distributions(model, target_input_ids, target_attention_mask, temperature, tw, special_tokens_map,
                                batch_size, verbose)
    return information_measure_cls(p, t)


def infolm(preds: Union[str, Sequence[str]], target: Union[str, Sequence[str]],
           model_name_or_path: Union[str, os.PathLike] = "bert-base-uncased", temperature: float = 0.25,
           information_measure: _ALLOWED_INFORMATION_MEASURE_LITERAL = "kl_divergence", idf: bool = True,
           alpha: Optional[float] = None, beta: Optional[float] = None,
           device: Optional[Union[str, torch.device]] = None, max_length: Optional[int] = None, batch_size: int = 64,
           num_threads: int = 0, verbose: bool = True, return_sentence_level_score: bool = False
           ) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    """Corpus InfoLM score (``F/text/infolm.py:540``).  ``model_name_or_path`` must be loadable offline."""
    tokenizer, model = _load_tokenizer_and_model(model_name_or_path, device)
    im = _InformationMeasure(information_measure, alpha, beta)
    max_length = max_length or model.config.max_length
    special = _get_special_tokens_map(tokenizer)
    pi, pa, ti, ta = _infolm_update(preds, target, tokenizer, max_length)
    scores = _infolm_compute(model, pi, pa, ti, ta, temperature, idf, im, special, batch_size, verbose)
    if return_sentence_level_score:
        return scores.mean(), scores
    return scores.mean()
