"""Text metrics, functional API (reference ``F/text/__init__.py``)."""
from torchmetrics_amd.functional.text.bleu import bleu_score, sacre_bleu_score
from torchmetrics_amd.functional.text.chrf import chrf_score
from torchmetrics_amd.functional.text.eed import extended_edit_distance
from torchmetrics_amd.functional.text.error_rates import (
    char_error_rate,
    edit_distance,
    match_error_rate,
    word_error_rate,
    word_information_lost,
    word_information_preserved,
)
from torchmetrics_amd.functional.text.perplexity import perplexity
from torchmetrics_amd.functional.text.rouge import rouge_score
from torchmetrics_amd.functional.text.squad import squad
from torchmetrics_amd.functional.text.ter import translation_edit_rate

__all__ = [
    "bleu_score",
    "char_error_rate",
    "chrf_score",
    "edit_distance",
    "extended_edit_distance",
    "match_error_rate",
    "perplexity",
    "rouge_score",
    "sacre_bleu_score",
    "squad",
    "translation_edit_rate",
    "word_error_rate",
    "word_information_lost",
    "word_information_preserved",
]

from torchmetrics_amd.utilities.imports import _TRANSFORMERS_AVAILABLE  # noqa: E402

if _TRANSFORMERS_AVAILABLE:
    from torchmetrics_amd.functional.text.bert import bert_score  # noqa: F401
    from torchmetrics_amd.functional.text.infolm import infolm  # noqa: F401

    __all__ += ["bert_score", "infolm"]
