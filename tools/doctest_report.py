#!/usr/bin/env python3
"""Replay every reference doctest (tests/golden/reference_doctests.json) and print a per-domain summary.

Usage: python tools/doctest_report.py [--only substring] [--show-failures N] [--json out.json]
"""
import argparse
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests.reference_doctests import (  # noqa: E402
    block_id,
    conditional_reason,
    domain_of,
    load_fixture,
    run_block,
    skip_reason,
)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--show-failures", type=int, default=0)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    data = load_fixture()
    stats = collections.defaultdict(lambda: collections.Counter())
    results = {}
    shown = 0
    t0 = time.time()
    for b in data["blocks"]:
        bid = block_id(b)
        if args.only and args.only not in bid:
            continue
        dom = domain_of(b)
        why = skip_reason(b)
        if why:
            stats[dom]["skipped"] += 1
            results[bid] = {"status": "skipped", "reason": why}
            continue
        try:
            failed, tried, report = run_block(b, data["modules"].get(b["file"], []))
        except Exception as err:  # noqa: BLE001
            failed, tried, report = 1, 1, repr(err)
        status = "passed" if failed == 0 else "failed"
        cond = conditional_reason(b)
        if failed and cond:
            status = "skipped"
            results[bid] = {"status": status, "reason": cond, "ours": report.strip().splitlines()[-1][:300]
                            if report.strip() else ""}
        else:
            results[bid] = {"status": status, "failed": failed, "tried": tried}
        stats[dom][status] += 1
        if failed and shown < args.show_failures:
            shown += 1
            print("=" * 100, "\n", bid, "\n", report[:3000])
    tot = collections.Counter()
    for dom in sorted(stats):
        c = stats[dom]
        tot.update(c)
        print(f"{dom:38s} passed {c['passed']:4d}  failed {c['failed']:4d}  skipped {c['skipped']:4d}")
    print(f"{'TOTAL':38s} passed {tot['passed']:4d}  failed {tot['failed']:4d}  skipped {tot['skipped']:4d}"
          f"   ({time.time() - t0:.0f} s)")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
