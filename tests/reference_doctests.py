"""Replay the reference's docstring examples (``tests/golden/reference_doctests.json``) against ``torchmetrics_amd``.

``import torchmetrics...`` inside an example resolves to the matching ``torchmetrics_amd`` module (a meta-path
alias installed for the run), each docstring runs in a namespace holding its module's top-level imports (as doctest
runs examples in the module globals), and outputs are compared like doctest with NORMALIZE_WHITESPACE + ELLIPSIS --
except that numbers are compared with a tolerance (the reference prints 4 decimals; our fp64 accumulations may move
the last digit), as doctest-plus's FLOAT_CMP does.

Used by ``tests/test_reference_doctests.py`` (pytest) and ``tools/doctest_report.py`` (per-domain summary).
"""
import contextlib
import doctest
import importlib
import importlib.abc
import importlib.util
import io
import json
import math
import re
import sys
import warnings
from pathlib import Path
from typing import Dict, List, Optional, Tuple

FIXTURE = Path(__file__).resolve().parent / "golden" / "reference_doctests.json"
_NUM = re.compile(r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?|nan|inf")


class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """``torchmetrics[.x.y]`` -> ``torchmetrics_amd[.x.y]``."""

    def find_spec(self, name, path=None, target=None):  # noqa: D102
        if name == "torchmetrics" or name.startswith("torchmetrics."):
            return importlib.util.spec_from_loader(name, self)
        return None

    def create_module(self, spec):  # noqa: D102
        return importlib.import_module("torchmetrics_amd" + spec.name[len("torchmetrics"):])

    def exec_module(self, module):  # noqa: D102
        pass


@contextlib.contextmanager
def reference_alias():
    saved = {k: v for k, v in sys.modules.items() if k == "torchmetrics" or k.startswith("torchmetrics.")}
    for k in saved:
        del sys.modules[k]
    # already-loaded modules answer directly (no loader run -> the import system does not rebind package attributes)
    ours = {k: v for k, v in sys.modules.items() if k == "torchmetrics_amd" or k.startswith("torchmetrics_amd.")}
    for k, v in ours.items():
        sys.modules["torchmetrics" + k[len("torchmetrics_amd"):]] = v
    # the loader binds a freshly loaded submodule on its (shared) package object: undo that for attributes that
    # were not modules (e.g. the function `dice` next to the module `dice`)
    attrs = {k: dict(vars(v)) for k, v in ours.items() if hasattr(v, "__path__")}
    finder = _AliasFinder()
    sys.meta_path.insert(0, finder)
    try:
        yield
    finally:
        sys.meta_path.remove(finder)
        for k in [k for k in sys.modules if k == "torchmetrics" or k.startswith("torchmetrics.")]:
            del sys.modules[k]
        sys.modules.update(saved)
        for k, before in attrs.items():
            pkg = sys.modules.get(k)
            for name, old in before.items():
                if pkg is not None and not isinstance(old, type(sys)) and vars(pkg).get(name) is not old:
                    setattr(pkg, name, old)


def _numbers_close(want: str, got: str, rtol: float, atol: float) -> bool:
    """Same text once numbers are masked, and pairwise-close numbers."""
    if _NUM.sub("#", want).split() != _NUM.sub("#", got).split():
        return False
    for a, b in zip(_NUM.findall(want), _NUM.findall(got)):
        fa, fb = float(a), float(b)
        if math.isnan(fa) and math.isnan(fb):
            continue
        if math.isinf(fa) or math.isinf(fb):
            if fa != fb:
                return False
            continue
        # the reference prints 4 decimals: half a unit of the last printed digit is rounding, not a difference
        digits = len(a.split(".")[1].split("e")[0].split("E")[0]) if "." in a else 0
        slack = 0.5 * 10 ** (-digits) if digits else 0.0
        if abs(fa - fb) > atol + slack + rtol * abs(fa):
            return False
    return True


class TolerantChecker(doctest.OutputChecker):
    def __init__(self, rtol: float = 1e-3, atol: float = 1e-4) -> None:
        self.rtol, self.atol = rtol, atol

    def check_output(self, want: str, got: str, optionflags: int) -> bool:  # noqa: D102
        flags = optionflags | doctest.NORMALIZE_WHITESPACE | doctest.ELLIPSIS
        if super().check_output(want, got, flags):
            return True
        return _numbers_close(want, got, self.rtol, self.atol)


def load_fixture() -> Dict:
    return json.loads(FIXTURE.read_text())


def block_id(b: Dict) -> str:
    name = b["name"] or "<module>"
    return f"{b['file'].replace('src/torchmetrics/', '')}::{name}"


def domain_of(b: Dict) -> str:
    parts = b["file"].split("/")
    return parts[2] if parts[2] != "functional" else "functional/" + parts[3].replace(".py", "")


def _importable(mod: str) -> bool:
    try:
        return importlib.util.find_spec(mod) is not None
    except (ImportError, ValueError):
        return False


def skip_reason(b: Dict) -> Optional[str]:
    """Why a docstring cannot run here at all (None: run it)."""
    src = "".join(e["source"] for e in b["examples"])
    if (b["skip"] and "MATPLOTLIB" in b["skip"] or ".plot(" in src) and not _importable("matplotlib"):
        return "plots need matplotlib (not installed; the reference skips these without it)"
    if b["skip"] and "always" in b["skip"]:
        return f"reference: {b['skip']}"
    return None


def conditional_reason(b: Dict) -> Optional[str]:
    """The reference skips this docstring in environments without an optional dependency (torchvision, pystoi,
    ...).  Many of those are dependencies of the reference only -- this package has native kernels instead -- so the
    examples are attempted; a failure is reported as a skip carrying this reason, not as a parity failure."""
    if b["skip"] and "MATPLOTLIB" not in b["skip"]:
        return f"reference: {b['skip']}"
    missing = [m for m in b.get("requires") or []
               if not _importable(m.split(">")[0].split("=")[0].split("<")[0].strip())]
    if missing:
        return f"reference requires {missing} (not installed here)"
    return None


def run_block(b: Dict, setup: List[str], checker: Optional[doctest.OutputChecker] = None) -> Tuple[int, int, str]:
    """Run one docstring's examples; returns (failures, tries, report)."""
    import torch

    globs: Dict = {"torch": torch}
    with reference_alias(), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        # doctest runs an example in its module's globals: start from our module at the same path
        mod_name = b["file"][len("src/"):-len(".py")].replace("/", ".")
        if mod_name.endswith(".__init__"):
            mod_name = mod_name[: -len(".__init__")]
        try:
            globs.update({k: v for k, v in vars(importlib.import_module(mod_name)).items() if not k.startswith("__")})
        except Exception:  # noqa: BLE001 - no module at that path
            pass
        for stmt in setup:
            try:
                exec(stmt, globs)  # noqa: S102 - the module's own top-level import lines
            except Exception:  # noqa: BLE001 - optional deps of the reference module
                pass
        examples = []
        for e in b["examples"]:
            opts = {doctest.OPTIONFLAGS_BY_NAME[k]: v for k, v in e["options"].items() if k in doctest.OPTIONFLAGS_BY_NAME}
            m = doctest.DocTestParser._EXCEPTION_RE.match(e["want"])
            examples.append(doctest.Example(e["source"], e["want"], exc_msg=m.group("msg") if m else None,
                                            lineno=e["line"], options=opts))
        test = doctest.DocTest(examples, globs, block_id(b), b["file"], b["line"], None)
        out = io.StringIO()
        runner = doctest.DocTestRunner(checker=checker or TolerantChecker(), optionflags=doctest.NORMALIZE_WHITESPACE
                                       | doctest.ELLIPSIS)
        torch.manual_seed(0)
        res = runner.run(test, out=out.write, clear_globs=True)
    return res.failed, res.attempted, out.getvalue()


doctest.register_optionflag("FLOAT_CMP")
