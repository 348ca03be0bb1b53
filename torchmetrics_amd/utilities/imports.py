"""Optional-dependency / version flags (parity: reference ``S/utilities/imports.py:24-68``).

``RequirementCache`` is re-implemented on ``importlib`` + ``packaging`` (no lightning-utilities dependency).
"""
import importlib.util
import shutil
import sys
from functools import lru_cache

from packaging.requirements import Requirement
from packaging.version import Version


class RequirementCache:
    """Lazy, truthy check that a requirement string (``"pkg>=1.0"``) or module is importable."""

    def __init__(self, requirement: str, module: str = None) -> None:
        self.requirement = requirement
        self.module = module

    @lru_cache(maxsize=None)  # noqa: B019
    def _check(self) -> bool:
        try:
            req = Requirement(self.requirement)
        except Exception:
            return importlib.util.find_spec(self.requirement) is not None
        name = self.module or req.name
        try:
            if importlib.util.find_spec(name) is None:
                return False
        except (ImportError, ValueError):
            return False
        if not req.specifier:
            return True
        try:
            from importlib.metadata import version

            ver = version(req.name)
        except Exception:
            try:
                ver = importlib.import_module(name).__version__
            except Exception:
                return False
        return Version(ver.split("+")[0]) in req.specifier or req.specifier.contains(ver, prereleases=True)

    def __bool__(self) -> bool:
        return self._check()

    def __str__(self) -> str:
        return f"Requirement {self.requirement!r} {'met' if self else 'not met'}"

    def __repr__(self) -> str:
        return self.__str__()


_PYTHON_VERSION = ".".join(map(str, sys.version_info[:3]))
_PYTHON_LOWER_3_8 = sys.version_info < (3, 8)
_TORCH_LOWER_2_0 = RequirementCache("torch<2.0.0")
_TORCH_GREATER_EQUAL_1_11 = RequirementCache("torch>=1.11.0")
_TORCH_GREATER_EQUAL_1_12 = RequirementCache("torch>=1.12.0")
_TORCH_GREATER_EQUAL_1_13 = RequirementCache("torch>=1.13.0")
_TORCH_GREATER_EQUAL_2_0 = RequirementCache("torch>=2.0.0")
_TORCH_GREATER_EQUAL_2_1 = RequirementCache("torch>=2.1.0")
_TORCH_GREATER_EQUAL_2_2 = RequirementCache("torch>=2.2.0")

_JIWER_AVAILABLE = RequirementCache("jiwer")
_NLTK_AVAILABLE = RequirementCache("nltk")
_ROUGE_SCORE_AVAILABLE = RequirementCache("rouge_score")
_BERTSCORE_AVAILABLE = RequirementCache("bert_score")
_SCIPY_AVAILABLE = RequirementCache("scipy")
_SCIPY_GREATER_EQUAL_1_8 = RequirementCache("scipy>=1.8.0")
_TORCH_FIDELITY_AVAILABLE = RequirementCache("torch_fidelity")
_LPIPS_AVAILABLE = RequirementCache("lpips")
_PYCOCOTOOLS_AVAILABLE = RequirementCache("pycocotools")
_TORCHVISION_AVAILABLE = RequirementCache("torchvision")
_TORCHVISION_GREATER_EQUAL_0_8 = RequirementCache("torchvision>=0.8.0")
_TORCHVISION_GREATER_EQUAL_0_13 = RequirementCache("torchvision>=0.13.0")
_TQDM_AVAILABLE = RequirementCache("tqdm")
_TRANSFORMERS_AVAILABLE = RequirementCache("transformers")
_TRANSFORMERS_GREATER_EQUAL_4_4 = RequirementCache("transformers>=4.4.0")
_TRANSFORMERS_GREATER_EQUAL_4_10 = RequirementCache("transformers>=4.10.0")
_PESQ_AVAILABLE = RequirementCache("pesq")
_GAMMATONE_AVAILABLE = RequirementCache("gammatone")
_TORCHAUDIO_AVAILABLE = RequirementCache("torchaudio")
_TORCHAUDIO_GREATER_EQUAL_0_10 = RequirementCache("torchaudio>=0.10.0")
_SACREBLEU_AVAILABLE = RequirementCache("sacrebleu")
_REGEX_AVAILABLE = RequirementCache("regex")
_PYSTOI_AVAILABLE = RequirementCache("pystoi")
_FAST_BSS_EVAL_AVAILABLE = RequirementCache("fast_bss_eval")
_MATPLOTLIB_AVAILABLE = RequirementCache("matplotlib")
_SCIENCEPLOT_AVAILABLE = RequirementCache("scienceplots")
_MULTIPROCESSING_AVAILABLE = RequirementCache("multiprocessing")
_XLA_AVAILABLE = RequirementCache("torch_xla")
_PIQ_GREATER_EQUAL_0_8 = RequirementCache("piq>=0.8.0")
_FASTER_COCO_EVAL_AVAILABLE = RequirementCache("faster_coco_eval")
_MECAB_AVAILABLE = RequirementCache("MeCab")
_MECAB_KO_AVAILABLE = RequirementCache("mecab_ko")
_MECAB_KO_DIC_AVAILABLE = RequirementCache("mecab_ko_dic")
_IPADIC_AVAILABLE = RequirementCache("ipadic")
_SENTENCEPIECE_AVAILABLE = RequirementCache("sentencepiece")
_SKLEARN_AVAILABLE = RequirementCache("scikit-learn", module="sklearn")

_LATEX_AVAILABLE: bool = shutil.which("latex") is not None
