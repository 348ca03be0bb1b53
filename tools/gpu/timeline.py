"""Per-dispatch timeline of a rocprofv3 run (kernel trace + HIP runtime trace, CSV): every HIP API call and every
kernel between two markers, on one clock, relative to the first timed kernel.  Usage:
python tools/gpu/timeline.py <dir> --kernel SUBSTR --skip N --count K
prints, for the K dispatches of kernels matching SUBSTR after the first N of them: host launch call (start, dur),
GPU start, GPU duration, idle gap before it, and the API calls around the region (memcpy / synchronize)."""
import csv
import glob
import sys


def main() -> None:
    d = sys.argv[1]
    sub = sys.argv[sys.argv.index("--kernel") + 1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1])
    count = int(sys.argv[sys.argv.index("--count") + 1])
    kt = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
    api = list(csv.DictReader(open(glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)[0])))
    kt.sort(key=lambda r: int(r["Start_Timestamp"]))
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    by_corr = {r["Correlation_Id"]: r for r in api}
    hits = [r for r in kt if sub in r["Kernel_Name"]]
    sel = hits[skip:skip + count]
    t0 = int(by_corr[sel[0]["Correlation_Id"]]["Start_Timestamp"]) if sel[0]["Correlation_Id"] in by_corr else int(
        sel[0]["Start_Timestamp"])
    t_end = int(sel[-1]["End_Timestamp"])
    # everything from the first timed launch call to 300 us after the last timed kernel
    ev = []
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 - 50_000 <= s <= t_end + 300_000 and r["Function"] not in ("hipGetDevice", "hipGetLastError",
                                                                       "hipStreamIsCapturing",
                                                                       "hipDevicePrimaryCtxGetState"):
            ev.append((s, "API", r["Function"], (e - s) / 1e3, r["Correlation_Id"]))
    prev_end = None
    for r in kt:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 - 50_000 <= s <= t_end + 300_000:
            name = r["Kernel_Name"].replace("void ", "").split("(")[0].split("<")[0][-40:]
            gap = (s - prev_end) / 1e3 if prev_end else 0.0
            prev_end = e
            ev.append((s, "GPU", name, (e - s) / 1e3, r["Correlation_Id"], gap))
    ev.sort()
    print(f"{'t(us)':>9} {'kind':4} {'what':42} {'dur(us)':>8} {'gap':>7} corr")
    for x in ev:
        gap = f"{x[5]:7.2f}" if len(x) > 5 else "       "
        print(f"{(x[0] - t0) / 1e3:9.2f} {x[1]:4} {x[2][:42]:42} {x[3]:8.2f} {gap} {x[4]}")
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]
    print(f"\n{len(sel)} timed kernels: sum {sum(durs):.1f} us, avg {sum(durs) / len(durs):.2f}, min {min(durs):.2f}, "
          f"max {max(durs):.2f}; first launch call -> last kernel end {(t_end - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
