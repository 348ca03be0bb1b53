"""Timeline of ONE call of a multi-kernel host function from a rocprofv3 run (kernel trace + HIP runtime trace,
CSV): the window from the end of the previous dispatch of an end-marker kernel to the end of the last one.  Prints
every dispatch in the window (host launch call start, GPU start, duration, GPU idle gap before it) and totals:
window, device busy, device idle, host-API time by function.  Usage:
python tools/gpu/compute_window.py <dir> --end SUBSTR [--nth K]   (K-th from last window, default 1)"""
import collections
import csv
import glob
import sys


def main() -> None:
    d = sys.argv[1]
    end = sys.argv[sys.argv.index("--end") + 1]
    nth = int(sys.argv[sys.argv.index("--nth") + 1]) if "--nth" in sys.argv else 1
    kt = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
    api = list(csv.DictReader(open(glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)[0])))
    kt.sort(key=lambda r: int(r["Start_Timestamp"]))
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    by_corr = {r["Correlation_Id"]: r for r in api}
    marks = [i for i, r in enumerate(kt) if end in r["Kernel_Name"]]
    hi, lo = marks[-nth], marks[-nth - 1]
    win = kt[lo + 1:hi + 1]
    w0 = int(kt[lo]["End_Timestamp"])
    w1 = int(kt[hi]["End_Timestamp"])
    busy = 0
    prev_end = w0
    print(f"{'launch_us':>10} {'gpu_start':>10} {'dur_us':>8} {'gap_us':>8}  kernel")
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        a = by_corr.get(r["Correlation_Id"])
        la = (int(a["Start_Timestamp"]) - w0) / 1e3 if a else float("nan")
        gap = max(0, s - prev_end)
        print(f"{la:10.1f} {(s - w0) / 1e3:10.1f} {(e - s) / 1e3:8.2f} {gap / 1e3:8.2f}  {r['Kernel_Name'][:90]}")
        busy += e - s
        prev_end = max(prev_end, e)
    fn = collections.Counter()
    cnt = collections.Counter()
    for a in api:
        s, e = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
        if w0 <= s <= w1:
            fn[a["Function"]] += e - s
            cnt[a["Function"]] += 1
    print(f"window {(w1 - w0) / 1e3:.1f} us, dispatches {len(win)}, device busy {busy / 1e3:.1f} us, "
          f"idle {(w1 - w0 - busy) / 1e3:.1f} us")
    for f, t in fn.most_common(12):
        print(f"  {f:40s} calls {cnt[f]:4d}  {t / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
