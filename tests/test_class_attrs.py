"""Class-level behaviour flags agree with the reference for every metric class.

``is_differentiable`` / ``higher_is_better`` / ``full_state_update`` and the plot bounds are read by users and by
trainers (checkpoint "best" selection uses ``higher_is_better``), so they are API.  The reference values come from
``tests/golden/reference_class_attrs.json`` (``tools/extract_reference_class_attrs.py``: parsed with ``ast`` from the
reference sources), resolved through the recorded base classes like Python's attribute lookup.
"""
import importlib
import json
from pathlib import Path

import pytest

FIXTURE = Path(__file__).resolve().parent / "golden" / "reference_class_attrs.json"
DATA = json.loads(FIXTURE.read_text())
_BY_NAME = {}
for _key in DATA:
    _BY_NAME.setdefault(_key.split(":")[1], []).append(_key)


def _base_key(name, module):
    keys = _BY_NAME.get(name, [])
    same = [k for k in keys if k.split(":")[0] == module]
    if same:
        return same[0]
    real = [k for k in keys if "_deprecated" not in k]
    return (real or keys or [None])[0]


def _resolve(key, attr, seen=()):
    """Reference value of ``attr`` on class ``key`` (left-to-right depth-first over recorded bases, as the MRO is
    for these single-inheritance-with-mixins trees); ``(False, None)`` when no recorded class assigns it."""
    if key is None or key in seen:
        return False, None
    entry = DATA[key]
    if attr in entry["attrs"]:
        return True, entry["attrs"][attr]
    for b in entry["bases"]:
        found, val = _resolve(_base_key(b, key.split(":")[0]), attr, seen + (key,))
        if found:
            return True, val
    return False, None


def _is_metric(key, seen=()):
    if key is None or key in seen:
        return False
    if key.endswith(":Metric"):
        return True
    return any(_is_metric(_base_key(b, key.split(":")[0]), seen + (key,)) for b in DATA[key]["bases"])


METRIC_CLASSES = sorted(k for k in DATA if _is_metric(k) and not k.split(":")[1].startswith("_")
                        and ".utilities." not in k)


def _ours(key):
    mod, name = key.split(":")
    module = importlib.import_module("torchmetrics_amd" + mod[len("torchmetrics"):])
    return getattr(module, name)


@pytest.mark.parametrize("key", METRIC_CLASSES)
def test_class_flags_match_reference(key):
    cls = _ours(key)
    diffs = []
    for attr in ("is_differentiable", "higher_is_better", "full_state_update", "plot_lower_bound", "plot_upper_bound",
                 "plot_legend_name"):
        found, want = _resolve(key, attr)
        if not found:
            continue
        got = getattr(cls, attr, "<missing>")
        if isinstance(want, float) and isinstance(got, (int, float)) and not isinstance(got, bool):
            same = float(got) == want
        else:
            same = got == want and type(got) is type(want)
        if not same:
            diffs.append(f"{attr}: reference {want!r}, ours {got!r}")
    assert not diffs, "; ".join(diffs)


def test_fixture_covers_the_metric_tree():
    assert len(METRIC_CLASSES) > 150
