"""Model-based text metrics: BERTScore and InfoLM (parity: reference ``S/text/bert.py``, ``S/text/infolm.py``).
Sentences are stored tokenised (``cat`` states of input ids / attention masks) so DDP gathers tensors, and the
encoder runs once at ``compute``."""
import os
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from torch.nn import Module

from torchmetrics_amd.functional.text._embedding import tokenize
from torchmetrics_amd.functional.text.bert import _DEFAULT_MODEL, bert_score
from torchmetrics_amd.functional.text.infolm import (
    _ALLOWED_INFORMATION_MEASURE_LITERAL,
    _get_special_tokens_map,
    _infolm_compute,
    _infolm_update,
    _InformationMeasure,
    _load_tokenizer_and_model,
)
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import dim_zero_cat
from torchmetrics_amd.utilities.imports import _TRANSFORMERS_AVAILABLE
from torchmetrics_amd.utilities.prints import rank_zero_warn


class _TokenStore(Metric):
    def _add_token_states(self) -> None:
        for name in ("preds_input_ids", "preds_attention_mask", "target_input_ids", "target_attention_mask"):
            self.add_state(name, [], dist_reduce_fx="cat")

    def _store(self, p: Dict[str, Tensor], t: Dict[str, Tensor]) -> None:
        self.preds_input_ids.append(p["input_ids"])
        self.preds_attention_mask.append(p["attention_mask"])
        self.target_input_ids.append(t["input_ids"])
        self.target_attention_mask.append(t["attention_mask"])

    def _stored(self, side: str) -> Dict[str, Tensor]:
        return {"input_ids": dim_zero_cat(getattr(self, f"{side}_input_ids")),
                "attention_mask": dim_zero_cat(getattr(self, f"{side}_attention_mask"))}


class BERTScore(_TokenStore):
    """BERTScore (``S/text/bert.py:54``)."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, model_name_or_path: Optional[str] = None, num_layers: Optional[int] = None,
                 all_layers: bool = False, model: Optional[Module] = None, user_tokenizer: Optional[Any] = None,
                 user_forward_fn: Optional[Callable[[Module, Dict[str, Tensor]], Tensor]] = None,
                 verbose: bool = False, idf: bool = False, device: Optional[Union[str, torch.device]] = None,
                 max_length: int = 512, batch_size: int = 64, num_threads: int = 0, return_hash: bool = False,
                 lang: str = "en", rescale_with_baseline: bool = False, baseline_path: Optional[str] = None,
                 baseline_url: Optional[str] = None, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.model_name_or_path = model_name_or_path or _DEFAULT_MODEL
        self.num_layers, self.all_layers, self.model = num_layers, all_layers, model
        self.user_forward_fn, self.verbose, self.idf = user_forward_fn, verbose, idf
        self.embedding_device, self.max_length, self.batch_size = device, max_length, batch_size
        self.num_threads, self.return_hash, self.lang = num_threads, return_hash, lang
        self.rescale_with_baseline, self.baseline_path, self.baseline_url = (rescale_with_baseline, baseline_path,
                                                                             baseline_url)
        if user_tokenizer:
            self.tokenizer, self.user_tokenizer = user_tokenizer, True
        else:
            if not _TRANSFORMERS_AVAILABLE:
                raise ModuleNotFoundError("`BERTScore` metric with default tokenizers requires `transformers`.")
            from transformers import AutoTokenizer

            if model_name_or_path is None:
                rank_zero_warn(
                    "The argument `model_name_or_path` was not specified while it is required when the default"
                    f" `transformers` model is used. It will use the default recommended model - {_DEFAULT_MODEL!r}."
                )
            self.tokenizer, self.user_tokenizer = AutoTokenizer.from_pretrained(self.model_name_or_path), False
        self._add_token_states()

    def update(self, preds: Union[str, Sequence[str]], target: Union[str, Sequence[str]]) -> None:
        preds = [preds] if isinstance(preds, str) else list(preds)
        target = [target] if isinstance(target, str) else list(target)
        p = tokenize(preds, self.tokenizer, self.max_length, own_tokenizer=self.user_tokenizer, truncation=False)
        t = tokenize(target, self.tokenizer, self.max_length, own_tokenizer=self.user_tokenizer, truncation=False)
        self._store(p, t)

    def compute(self) -> Dict[str, Union[Tensor, List[float], str]]:
        return bert_score(
            preds=self._stored("preds"), target=self._stored("target"), model_name_or_path=self.model_name_or_path,
            num_layers=self.num_layers, all_layers=self.all_layers, model=self.model,
            user_tokenizer=self.tokenizer if self.user_tokenizer else None, user_forward_fn=self.user_forward_fn,
            verbose=self.verbose, idf=self.idf, device=self.embedding_device, max_length=self.max_length,
            batch_size=self.batch_size, num_threads=self.num_threads, return_hash=self.return_hash, lang=self.lang,
            rescale_with_baseline=self.rescale_with_baseline, baseline_path=self.baseline_path,
            baseline_url=self.baseline_url,
        )

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        val = val or {k: v.mean() for k, v in self.compute().items() if isinstance(v, Tensor)}
        return self._plot(val, ax)


class InfoLM(_TokenStore):
    """InfoLM (``S/text/infolm.py:41``)."""

    is_differentiable = False
    higher_is_better = True

    def __init__(self, model_name_or_path: Union[str, os.PathLike] = "bert-base-uncased", temperature: float = 0.25,
                 information_measure: _ALLOWED_INFORMATION_MEASURE_LITERAL = "kl_divergence", idf: bool = True,
                 alpha: Optional[float] = None, beta: Optional[float] = None,
                 device: Optional[Union[str, torch.device]] = None, max_length: Optional[int] = None,
                 batch_size: int = 64, num_threads: int = 0, verbose: bool = True,
                 return_sentence_level_score: bool = False, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.model_name_or_path, self.temperature = model_name_or_path, temperature
        self.information_measure, self.idf, self.alpha, self.beta = information_measure, idf, alpha, beta
        self.embedding_device = torch.device(device or "cpu")
        self.batch_size, self.num_threads, self.verbose = batch_size, num_threads, verbose
        self.return_sentence_level_score = return_sentence_level_score
        self.tokenizer, self.model = _load_tokenizer_and_model(model_name_or_path, self.embedding_device)
        self.information_measure_cls = _InformationMeasure(information_measure, alpha, beta)
        self.max_length = max_length or self.model.config.max_length
        self.special_tokens_map = _get_special_tokens_map(self.tokenizer)
        self._add_token_states()

    def update(self, preds: Union[str, Sequence[str]], target: Union[str, Sequence[str]]) -> None:
        pi, pa, ti, ta = _infolm_update(preds, target, self.tokenizer, self.max_length)
        self._store({"input_ids": pi, "attention_mask": pa}, {"input_ids": ti, "attention_mask": ta})

    def compute(self) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        p, t = self._stored("preds"), self._stored("target")
        scores = _infolm_compute(self.model, p["input_ids"].cpu(), p["attention_mask"].cpu(), t["input_ids"].cpu(),
                                 t["attention_mask"].cpu(), self.temperature, self.idf, self.information_measure_cls,
                                 self.special_tokens_map, self.batch_size, self.verbose)
        if self.return_sentence_level_score:
            return scores.mean(), scores
        return scores.mean()

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)
