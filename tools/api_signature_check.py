#!/usr/bin/env python3
"""Compare constructor / function parameter names and order of every public reference class and functional with
``torchmetrics_amd`` (reference parsed with ``ast``, ours with ``inspect``).  Prints mismatches; exit 1 if any.

Usage: python tools/api_signature_check.py [--ref /root/reference]
"""
import argparse
import ast
import importlib
import inspect
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def ref_signatures(ref: Path):
    out = {}
    for path in (ref / "src" / "torchmetrics").rglob("*.py"):
        rel = path.relative_to(ref / "src").with_suffix("")
        mod = ".".join(rel.parts).replace(".__init__", "")
        tree = ast.parse(path.read_text())
        for node in tree.body:
            if isinstance(node, ast.ClassDef) and not node.name.startswith("_"):
                for sub in node.body:
                    if isinstance(sub, ast.FunctionDef) and sub.name in ("__init__", "__new__"):
                        args = [a.arg for a in sub.args.args[1:]] + [a.arg for a in sub.args.kwonlyargs]
                        out[(mod, node.name)] = args
            elif isinstance(node, ast.FunctionDef) and not node.name.startswith("_") and ".functional." in f".{mod}.":
                out[(mod, node.name)] = [a.arg for a in node.args.args] + [a.arg for a in node.args.kwonlyargs]
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    bad = 0
    checked = 0
    for (mod, name), ref_args in sorted(ref_signatures(Path(args.ref)).items()):
        ours_mod = "torchmetrics_amd" + mod[len("torchmetrics"):]
        try:
            obj = getattr(importlib.import_module(ours_mod), name)
        except (ImportError, AttributeError):
            continue
        target = obj.__new__ if "__new__" in vars(obj) else (obj.__init__ if inspect.isclass(obj) else obj)
        try:
            params = [p.name for p in inspect.signature(target).parameters.values()
                      if p.kind not in (p.VAR_POSITIONAL, p.VAR_KEYWORD)]
        except (TypeError, ValueError):
            continue
        if inspect.isclass(obj) and params and params[0] in ("self", "cls"):
            params = params[1:]
        ref_named = [a for a in ref_args if a not in ("self", "cls")]
        checked += 1
        if params[: len(ref_named)] != ref_named:
            bad += 1
            print(f"{mod}.{name}\n   ref : {ref_named}\n   ours: {params}")
    print(f"checked {checked}, mismatched {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
