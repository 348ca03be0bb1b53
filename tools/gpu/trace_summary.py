"""Summarise a rocprofv3 kernel_trace.csv: per kernel (short name, grid) the call count and median duration; with
--per-call N, the kernels (and total device time) per call of the timed loop.  Usage:
python tools/gpu/trace_summary.py <dir> [--match SUBSTR] [--calls N]"""
import collections
import csv
import glob
import sys


def main() -> None:
    d = sys.argv[1]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    calls = int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 0
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    gx = next(k for k in rows[0] if k.startswith("Grid_Size"))
    by = collections.defaultdict(list)
    for x in rows:
        n = x["Kernel_Name"]
        if match and match not in n:
            continue
        short = n.replace("void ", "").replace("tm_amd::(anonymous namespace)::", "").replace(
            "at::native::(anonymous namespace)::", "").split("(")[0][:70]
        by[(short, x[gx])].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000)
    tot = 0.0
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        tot += sum(v)
        print(f"{k[0]:72s} grid={k[1]:>8s} n={len(v):5d} med={v[len(v) // 2]:8.2f}us sum={sum(v):10.1f}us")
    if calls:
        print(f"total {tot:.1f} us over {calls} calls: {tot / calls:.2f} us / call")


if __name__ == "__main__":
    main()
