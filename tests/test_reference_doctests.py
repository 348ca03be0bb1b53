"""Golden values: every ``>>>`` example of the reference's docstrings, replayed against ``torchmetrics_amd``.

The examples (inputs and expected outputs) are extracted from the reference once by
``tools/extract_reference_doctests.py`` into ``tests/golden/reference_doctests.json``; ``tests/reference_doctests.py``
replays a docstring's examples in order (``torchmetrics`` imports resolved to this package) and compares outputs
like doctest, numbers within the reference's printed precision.  Docstrings the reference itself skips without an
optional dependency (``__doctest_skip__`` / ``__doctest_requires__``: torchvision, pystoi, ...) are still attempted --
most of those dependencies are the reference's, not ours -- and only a failure there is reported as a skip with that
reason; plots (matplotlib not installed) are skipped.  Each test id carries the docstring's location.
The ROCm kernels are pinned to these host paths by the GPU suite (kernel vs host implementation of the same op).
"""
import pytest

from tests.reference_doctests import block_id, conditional_reason, load_fixture, run_block, skip_reason

_DATA = load_fixture()


@pytest.mark.parametrize("block", _DATA["blocks"], ids=[block_id(b) for b in _DATA["blocks"]])
def test_reference_doctest(block):
    why = skip_reason(block)
    if why:
        pytest.skip(why)
    failed, tried, report = run_block(block, _DATA["modules"].get(block["file"], []))
    assert tried > 0
    cond = conditional_reason(block)
    if failed and cond:
        pytest.skip(f"{cond}; ours: {report.strip().splitlines()[-1][:200] if report.strip() else 'failed'}")
    assert failed == 0, f"{block['file']}:{block['line']}\n{report}"
