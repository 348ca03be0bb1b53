#!/usr/bin/env python3
"""Extract the reference metrics' class-level attributes into a JSON fixture (parsed with ``ast``, never imported).

Every ``Metric`` subclass in the reference declares behaviour flags as class attributes -- ``is_differentiable``,
``higher_is_better``, ``full_state_update``, ``plot_lower_bound`` / ``plot_upper_bound`` / ``plot_legend_name``.
Users (and Lightning) read them, so they are API.  This tool records, per ``module:Class``, the explicitly assigned
literal values and the base-class names; ``tests/test_class_attrs.py`` resolves inheritance through the recorded
bases and checks ``torchmetrics_amd``'s classes agree.

Usage: ``python tools/extract_reference_class_attrs.py [--ref /root/reference]`` ->
``tests/golden/reference_class_attrs.json``.
"""
import argparse
import ast
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
ATTRS = ("is_differentiable", "higher_is_better", "full_state_update", "plot_lower_bound", "plot_upper_bound",
         "plot_legend_name")


def _literal(node):
    try:
        return True, ast.literal_eval(node)
    except ValueError:
        return False, None


def extract(ref: Path) -> dict:
    out = {}
    for path in sorted((ref / "src" / "torchmetrics").rglob("*.py")):
        mod = str(path.relative_to(ref / "src"))[:-3].replace("/", ".")
        if mod.endswith(".__init__"):
            mod = mod[: -len(".__init__")]
        for node in ast.parse(path.read_text()).body:
            if not isinstance(node, ast.ClassDef):
                continue
            attrs = {}
            for stmt in node.body:
                target, value = None, None
                if isinstance(stmt, ast.AnnAssign) and isinstance(stmt.target, ast.Name) and stmt.value is not None:
                    target, value = stmt.target.id, stmt.value
                elif isinstance(stmt, ast.Assign) and len(stmt.targets) == 1 and isinstance(stmt.targets[0], ast.Name):
                    target, value = stmt.targets[0].id, stmt.value
                if target in ATTRS:
                    ok, val = _literal(value)
                    if ok:
                        attrs[target] = val
            bases = [ast.unparse(b).split(".")[-1] for b in node.bases]
            out[f"{mod}:{node.name}"] = {"bases": bases, "attrs": attrs}
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=str(ROOT / "tests" / "golden" / "reference_class_attrs.json"))
    args = ap.parse_args()
    data = extract(Path(args.ref))
    Path(args.out).write_text(json.dumps(data, indent=0, sort_keys=True))
    print(f"{len(data)} classes -> {args.out}")


if __name__ == "__main__":
    main()
