#!/usr/bin/env python3
"""Extract the reference's doctest examples (inputs + expected outputs) into a JSON fixture.

The reference is tested with ``--doctest-modules --doctest-plus`` (``pyproject.toml``): every ``>>>`` example in its
docstrings is a golden value.  This tool parses (never imports) ``src/torchmetrics/**/*.py`` with ``ast`` and
``doctest.DocTestParser`` and writes ``tests/golden/reference_doctests.json``:

    {"modules": {"src/torchmetrics/...py": ["import torch", ...]},   # top-level imports (doctests run in globals)
     "blocks": [{"file": "src/torchmetrics/...py", "name": "Class.method", "line": 123,
      "skip": "reason" | null,                  # __doctest_skip__ / __doctest_requires__ of the module
      "examples": [{"source": ..., "want": ..., "line": ..., "options": {...}}]}]

The fixture is committed; ``tests/test_reference_doctests.py`` replays it against ``torchmetrics_amd`` without
needing the reference tree.  Usage: ``python tools/extract_reference_doctests.py [--ref /root/reference]``.
"""
import argparse
import ast
import doctest
import fnmatch
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _module_meta(tree: ast.Module):
    skips, requires, imports = [], {}, []
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            imports.append(ast.unparse(node))
        elif isinstance(node, ast.If):  # e.g. `if not _MATPLOTLIB_AVAILABLE: __doctest_skip__ = [...]`
            for sub in node.body + node.orelse:
                if isinstance(sub, ast.Assign):
                    _collect(sub, skips, requires, conditional=ast.unparse(node.test))
        elif isinstance(node, ast.Assign):
            _collect(node, skips, requires, conditional=None)
    return skips, requires, imports


def _collect(node: ast.Assign, skips: list, requires: dict, conditional) -> None:
    for tgt in node.targets:
        if not isinstance(tgt, ast.Name):
            continue
        try:
            val = ast.literal_eval(node.value)
        except ValueError:
            continue
        if tgt.id == "__doctest_skip__":
            skips.extend((p, conditional) for p in (val if isinstance(val, (list, tuple)) else [val]))
        elif tgt.id == "__doctest_requires__" and isinstance(val, dict):
            for pats, mods in val.items():
                for p in (pats if isinstance(pats, tuple) else (pats,)):
                    requires[p] = list(mods) if isinstance(mods, (list, tuple)) else [mods]


def _docstrings(tree: ast.Module):
    """(qualified name, docstring, line) of the module, its classes, functions and methods."""
    doc = ast.get_docstring(tree, clean=False)
    if doc:
        yield "", doc, 1
    stack = [(n, "") for n in tree.body]
    while stack:
        node, prefix = stack.pop(0)
        if isinstance(node, (ast.ClassDef, ast.FunctionDef, ast.AsyncFunctionDef)):
            name = f"{prefix}{node.name}"
            doc = ast.get_docstring(node, clean=False)
            if doc:
                yield name, doc, node.body[0].lineno
            if isinstance(node, ast.ClassDef):
                stack.extend((c, f"{name}.") for c in node.body)


def extract(ref: Path) -> dict:
    doctest.register_optionflag("FLOAT_CMP")  # doctest-plus flag used by a few reference examples
    blocks, modules = [], {}
    parser = doctest.DocTestParser()
    for path in sorted((ref / "src" / "torchmetrics").rglob("*.py")):
        tree = ast.parse(path.read_text())
        skips, requires, imports = _module_meta(tree)
        rel = str(path.relative_to(ref))
        modules[rel] = imports
        for name, doc, line in _docstrings(tree):
            try:
                examples = parser.get_examples(doc)
            except ValueError:
                continue
            if not examples:
                continue
            skip = None
            for pat, cond in skips:
                if fnmatch.fnmatch(name, pat) or fnmatch.fnmatch(f"{path.stem}.{name}", pat):
                    skip = f"__doctest_skip__ ({'if ' + cond if cond else 'always'})"
            for pat, mods in requires.items():
                if fnmatch.fnmatch(name, pat) or name.startswith(pat + "."):
                    skip = skip or f"__doctest_requires__ {mods}"
            blocks.append({
                "file": rel, "name": name, "line": line, "skip": skip,
                "requires": next((m for p, m in requires.items()
                                  if fnmatch.fnmatch(name, p) or name.startswith(p + ".")), []),
                "examples": [{"source": e.source, "want": e.want, "line": line + e.lineno,
                              "options": {doctest.OPTIONFLAGS_BY_NAME and next(
                                  (n for n, f in doctest.OPTIONFLAGS_BY_NAME.items() if f == k), str(k)): v
                                  for k, v in e.options.items()}} for e in examples],
            })
    return {"modules": {k: v for k, v in modules.items() if any(b["file"] == k for b in blocks)}, "blocks": blocks}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=str(ROOT / "tests" / "golden" / "reference_doctests.json"))
    args = ap.parse_args()
    data = extract(Path(args.ref))
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(data, indent=0))
    n_ex = sum(len(b["examples"]) for b in data["blocks"])
    print(f"{len(data['blocks'])} docstrings, {n_ex} examples -> {args.out}")


if __name__ == "__main__":
    main()
