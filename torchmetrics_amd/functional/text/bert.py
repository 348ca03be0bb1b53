"""BERTScore (reference ``F/text/bert.py``).

Contextual token embeddings come from a HuggingFace encoder (or a user model + forward function); the metric core is
batched greedy matching: per pair ``cos[p, r]`` = normalised-embedding GEMM (vendor MFMA GEMM through ``torch.matmul``),
precision = idf-weighted mean over prediction tokens of ``max_r cos``, recall likewise over reference tokens.  All
pairs of a batch (and all layers with ``all_layers=True``) are one batched GEMM + two ``amax`` reductions.

No network here: ``model_name_or_path`` must be a local directory (or pass ``model`` + ``user_tokenizer``); baseline
rescaling reads ``baseline_path`` (a URL download is refused).
"""
import csv
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from torch.nn import Module

from torchmetrics_amd import ops
from torchmetrics_amd.functional.text._embedding import idf_table, idf_weights, run_sorted, tokenize
from torchmetrics_amd.utilities.imports import _TQDM_AVAILABLE, _TRANSFORMERS_AVAILABLE
from torchmetrics_amd.utilities.prints import rank_zero_warn

_DEFAULT_MODEL = "roberta-large"


def _process_attention_mask_for_special_tokens(attention_mask: Tensor) -> Tensor:
    """Zero the first ([CLS]) and last valid ([SEP]) position of every row."""
    m = attention_mask.clone()
    m[:, 0] = 0
    last = torch.cumsum(attention_mask.float() - 0.1, dim=-1).argmax(-1)
    m[torch.arange(m.size(0)), last] = 0
    return m


def _embed(model: Module, input_ids: Tensor, attention_mask: Tensor, weights: Tensor, device: torch.device,
           num_layers: Optional[int], all_layers: bool, batch_size: int, verbose: bool,
           user_forward_fn: Optional[Callable]) -> Tuple[Tensor, Tensor]:
    """(normalised masked embeddings [N, L, S, D], normalised token weights [N, S]) in original row order."""
    proc = _process_attention_mask_for_special_tokens(attention_mask)
    w = weights * proc
    w = w / w.sum(-1, keepdim=True)

    def fn(rows: Tensor, ln: int) -> Tensor:
        ids = input_ids[rows, :ln].to(device)
        am = attention_mask[rows, :ln].to(device)
        with torch.no_grad():
            if all_layers:
                if user_forward_fn is not None:
                    raise ValueError("The option `all_layers=True` can be used only with default `transformers` models.")
                hs = model(ids, am, output_hidden_states=True).hidden_states
                out = torch.stack(list(hs), dim=1)
            elif user_forward_fn is not None:
                out = user_forward_fn(model, {"input_ids": ids, "attention_mask": am})
                if out.dim() != 3 or out.shape[0] != ids.shape[0] or out.shape[1] != ids.shape[1]:
                    raise ValueError(
                        "The model output must be `Tensor` of a shape `[batch_size, seq_len, model_dim]` "
                        f"i.e. [{ids.shape[0]}, {ids.shape[1]}. , `model_dim`], but got {out.shape}."
                    )
                out = out.unsqueeze(1)
            else:
                hs = model(ids, am, output_hidden_states=True).hidden_states
                out = hs[num_layers if num_layers is not None else -1].unsqueeze(1)
        out = out / out.norm(dim=-1, keepdim=True)
        out = out * proc[rows, :ln].to(out)[:, None, :, None]
        return out.transpose(1, 2)  # [rows, S, L, D] so run_sorted pads the token dim

    emb = run_sorted(attention_mask, batch_size, fn, verbose).transpose(1, 2)
    return emb, w[:, : emb.shape[2]].to(emb.device)


def _greedy_match(pe: Tensor, te: Tensor, pw: Tensor, tw: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """Batched greedy matching: pe [N, L, P, D], te [N, L, R, D] -> precision / recall / f1 [N, L].

    ROCm: one MFMA GEMM over all N * L pairs whose epilogue keeps only the row / column maxima of the token
    similarities (``ops.gemm_row_col_max``); the reference materialises the [N, L, P, R] cosine tensor
    (``F/text/bert.py:134-167``)."""
    n, nl, p, d = pe.shape
    r = te.shape[2]
    if pe.is_cuda and not (pe.requires_grad or te.requires_grad) and n * nl * p * r > 0:
        # ROCm: no [N, L, P, R] tensor -- sentence-length pairs (<= 128 tokens a side) on the per-pair 64 x 64
        # super-tile kernel, longer ones on the 128 x 128 MFMA GEMM with the row / column max epilogue
        # 16-bit embeddings (a bf16 / fp16 model: the reference's einsum runs in that dtype) stay 16-bit: the 16-bit
        # matrix cores, no fp32 upcast pass
        h16 = pe.dtype in (torch.bfloat16, torch.float16) and te.dtype == pe.dtype
        x = pe.reshape(n * nl, p, d)
        y = te.reshape(n * nl, r, d)
        x, y = (x.contiguous(), y.contiguous()) if h16 else (x.float().contiguous(), y.float().contiguous())
        if p <= 128 and r <= 128:
            rmax, cmax = ops.bert_rowcol_max(x, y)
        elif h16 or d % 4 == 0:
            rmax, cmax = ops.gemm_row_col_max(x, y)
            if h16:  # (the similarities in the embeddings' dtype, as the bert_rowcol_max path rounds them)
                rmax, cmax = rmax.to(pe.dtype).float(), cmax.to(pe.dtype).float()
        else:
            rmax = cmax = None
    else:
        rmax = cmax = None
    if rmax is not None:
        precision = (rmax.reshape(n, nl, p) * pw[:, None, :].float()).sum(-1)
        recall = (cmax.reshape(n, nl, r) * tw[:, None, :].float()).sum(-1)
        f1 = (2 * precision * recall / (precision + recall)).nan_to_num(0.0)
        return precision, recall, f1
    cos = torch.matmul(pe, te.transpose(-1, -2))  # [N, L, P, R]
    precision = (cos.amax(dim=3) * pw[:, None, :].to(cos)).sum(-1)
    recall = (cos.amax(dim=2) * tw[:, None, :].to(cos)).sum(-1)
    f1 = (2 * precision * recall / (precision + recall)).nan_to_num(0.0)
    return precision, recall, f1


def _load_baseline(lang: str = "en", model_name_or_path: Optional[str] = None, baseline_path: Optional[str] = None,
                   baseline_url: Optional[str] = None) -> Optional[Tensor]:
    if baseline_path:
        with open(baseline_path) as fh:
            rows = [[float(x) for x in row] for i, row in enumerate(csv.reader(fh)) if i > 0]
        return torch.tensor(rows)[:, 1:]
    if baseline_url or (lang and model_name_or_path):
        raise OSError("BERTScore baseline download is not possible without network access; pass `baseline_path`.")
    rank_zero_warn("Baseline was not successfully loaded. No baseline is going to be used.")
    return None


def _rescale_metrics_with_baseline(precision: Tensor, recall: Tensor, f1_score: Tensor, baseline: Tensor,
                                   num_layers: Optional[int] = None, all_layers: bool = False
                                   ) -> Tuple[Tensor, Tensor, Tensor]:
    if num_layers is None and all_layers is False:
        num_layers = -1
    m = torch.stack([precision, recall, f1_score], dim=-1)
    b = baseline.unsqueeze(1) if all_layers else baseline[num_layers]
    m = (m - b.to(m)) / (1 - b.to(m))
    return m[..., 0], m[..., 1], m[..., 2]


def _get_hash(model_name_or_path: Optional[str] = None, num_layers: Optional[int] = None, idf: bool = False) -> str:
    return f"{model_name_or_path}_L{num_layers}{'_idf' if idf else '_no-idf'}"


def _load_default(model_name_or_path: Optional[str]) -> Tuple[Any, Module]:
    if not _TRANSFORMERS_AVAILABLE:
        raise ModuleNotFoundError("`bert_score` metric with default models requires `transformers` package be installed.")
    from transformers import AutoModel, AutoTokenizer

    if model_name_or_path is None:
        rank_zero_warn(
            "The argument `model_name_or_path` was not specified while it is required when default `transformers` model"
            f" are used. It is, therefore, used the default recommended model - {_DEFAULT_MODEL}."
        )
    name = model_name_or_path or _DEFAULT_MODEL
    return AutoTokenizer.from_pretrained(name), AutoModel.from_pretrained(name)


def bert_score(preds: Union[str, Sequence[str], Dict[str, Tensor]], target: Union[str, Sequence[str], Dict[str, Tensor]],
               model_name_or_path: Optional[str] = None, num_layers: Optional[int] = None, all_layers: bool = False,
               model: Optional[Module] = None, user_tokenizer: Any = None,
               user_forward_fn: Optional[Callable[[Module, Dict[str, Tensor]], Tensor]] = None, verbose: bool = False,
               idf: bool = False, device: Optional[Union[str, torch.device]] = None, max_length: int = 512,
               batch_size: int = 64, num_threads: int = 0, return_hash: bool = False, lang: str = "en",
               rescale_with_baseline: bool = False, baseline_path: Optional[str] = None,
               baseline_url: Optional[str] = None) -> Dict[str, Union[Tensor, List[float], str]]:
    """BERTScore precision / recall / F1 per sentence pair (``F/text/bert.py:253``)."""
    if isinstance(preds, str):
        preds = [preds]
    if isinstance(target, str):
        target = [target]
    if len(preds) != len(target):
        raise ValueError("Number of predicted and reference sententes must be the same!")
    if not isinstance(preds, (list, dict)):
        preds = list(preds)
    if not isinstance(target, (list, dict)):
        target = list(target)
    if verbose and not _TQDM_AVAILABLE:
        raise ModuleNotFoundError("An argument `verbose = True` requires `tqdm` package be installed.")
    if model is None:
        tokenizer, model = _load_default(model_name_or_path)
    else:
        tokenizer = user_tokenizer
    model.eval()
    dev = torch.device(device) if device is not None else next(model.parameters()).device
    model.to(dev)
    try:
        if num_layers and num_layers > model.config.num_hidden_layers:
            raise ValueError(
                f"num_layers={num_layers} is forbidden for {model_name_or_path}."
                f" Please use num_layers <= {model.config.num_hidden_layers}"
            )
    except AttributeError:
        rank_zero_warn("It was not possible to retrieve the parameter `num_layers` from the model specification.")

    if all(isinstance(t, list) and len(t) == 0 for t in (preds, target)):
        rank_zero_warn("Predictions and references are empty.")
        out: Dict[str, Any] = {"precision": [0.0], "recall": [0.0], "f1": [0.0]}
        if return_hash:
            out["hash"] = _get_hash(model_name_or_path, num_layers, idf)
        return out
    baseline = _load_baseline(lang, model_name_or_path, baseline_path, baseline_url) if rescale_with_baseline else None

    if all(isinstance(t, list) and len(t) > 0 and isinstance(t[0], str) for t in (preds, target)):
        if tokenizer is None:
            raise ValueError("A tokenizer is required for string inputs (pass `user_tokenizer` with `model`).")
        t_tok = tokenize(target, tokenizer, max_length)  # HF call convention, as the reference's TextDataset
        p_tok = tokenize(preds, tokenizer, max_length)
    elif all(isinstance(t, dict) and isinstance(t.get("input_ids"), Tensor) for t in (preds, target)):
        t_tok = {"input_ids": target["input_ids"], "attention_mask": target["attention_mask"]}
        p_tok = {"input_ids": preds["input_ids"], "attention_mask": preds["attention_mask"]}
    else:
        raise ValueError("Invalid input provided.")

    if idf:
        table, default = idf_table(t_tok["input_ids"])
        tw, pw = idf_weights(t_tok["input_ids"], table, default), idf_weights(p_tok["input_ids"], table, default)
    else:
        tw, pw = t_tok["attention_mask"].float(), p_tok["attention_mask"].float()
    te, tws = _embed(model, t_tok["input_ids"], t_tok["attention_mask"], tw, dev, num_layers, all_layers, batch_size,
                     verbose, user_forward_fn)
    pe, pws = _embed(model, p_tok["input_ids"], p_tok["attention_mask"], pw, dev, num_layers, all_layers, batch_size,
                     verbose, user_forward_fn)
    precision, recall, f1 = _greedy_match(pe, te, pws, tws)  # [N, L]
    precision, recall, f1 = (x.transpose(0, 1).squeeze(0) if not all_layers else x.transpose(0, 1)
                             for x in (precision, recall, f1))
    if baseline is not None:
        precision, recall, f1 = _rescale_metrics_with_baseline(precision, recall, f1, baseline, num_layers, all_layers)
    res: Dict[str, Any] = {"precision": precision.cpu(), "recall": recall.cpu(), "f1": f1.cpu()}
    if return_hash:
        res["hash"] = _get_hash(model_name_or_path, num_layers, idf)
    return res
