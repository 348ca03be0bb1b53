"""The value layer of ``utilities.plot`` (what gets drawn), testable without matplotlib."""
import pytest
import torch

from torchmetrics_amd.utilities.plot import _confmat_panels, _curve_series, _get_col_row_split, _series_of


def test_series_single_vector_dict_history():
    s, steps = _series_of(torch.tensor(0.5))
    assert steps == 0 and len(s) == 1 and s[0].y.tolist() == [0.5] and not s[0].line
    s, steps = _series_of(torch.tensor([0.1, 0.2, 0.3]), legend_name="Class")
    assert [x.label for x in s] == ["Class 0", "Class 1", "Class 2"] and steps == 0
    s, steps = _series_of({"a": torch.tensor(1.0), "b": torch.tensor([1.0, 2.0, 3.0])})
    assert s[0].label == "a" and s[1].line and steps == 3
    hist = [torch.tensor([0.1, 0.9]), torch.tensor([0.2, 0.8]), torch.tensor([0.3, 0.7])]
    s, steps = _series_of(hist)
    assert steps == 3 and len(s) == 2 and s[1].y.tolist() == pytest.approx([0.9, 0.8, 0.7])
    s, steps = _series_of([{"x": torch.tensor(1.0)}, {"x": torch.tensor(2.0)}])
    assert steps == 2 and s[0].y.tolist() == [1.0, 2.0]
    with pytest.raises(ValueError):
        _series_of(3.0)


def test_confmat_panels_and_grid():
    p = _confmat_panels(torch.arange(9).reshape(3, 3), ["a", "b", "c"])
    assert len(p) == 1 and p[0].ticks == ["a", "b", "c"] and p[0].matrix[2, 1] == 7
    with pytest.raises(ValueError):
        _confmat_panels(torch.zeros(3, 3), ["a"])
    p = _confmat_panels(torch.zeros(5, 2, 2), None)
    assert [x.title for x in p] == [f"Label {i}" for i in range(5)]
    assert _get_col_row_split(5) == (2, 3) and _get_col_row_split(9) == (3, 3) and _get_col_row_split(7) == (3, 3)


def test_curve_series():
    x, y = torch.linspace(0, 1, 5), torch.linspace(0, 1, 5) ** 2
    s = _curve_series((x, y, x), torch.tensor(0.75), None)
    assert s[0].label == "AUC=0.750"
    s = _curve_series(([x, x], [y, y]), torch.tensor([0.5, 0.25]), "cls")
    assert [z.label for z in s] == ["cls_0 AUC=0.500", "cls_1 AUC=0.250"]
    with pytest.raises(ValueError):
        _curve_series((x,), None, None)
