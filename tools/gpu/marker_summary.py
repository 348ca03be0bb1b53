"""roctx ranges vs the HIP launches inside them (rocprofv3 --marker-trace --hip-runtime-trace --kernel-trace, CSV):
for every range, the hipLaunchKernel calls that started inside it and the kernels those launches produced (matched
by correlation id).  Usage: python tools/gpu/marker_summary.py <dir> [--match RANGE_SUBSTR]"""
import csv
import glob
import sys


def main() -> None:
    d = sys.argv[1]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    one = lambda pat: list(csv.DictReader(open(glob.glob(f"{d}/**/*{pat}", recursive=True)[0])))  # noqa: E731
    marks = [r for r in one("marker_api_trace.csv") if match in r["Function"]]
    api = [r for r in one("hip_api_trace.csv") if r["Function"].startswith(("hipLaunchKernel", "hipExtLaunch",
                                                                            "hipModuleLaunch"))]
    kern = {r["Correlation_Id"]: r for r in one("kernel_trace.csv")}
    inside_total = 0
    for m in sorted(marks, key=lambda r: int(r["Start_Timestamp"])):
        s, e = int(m["Start_Timestamp"]), int(m["End_Timestamp"])
        launches = [a for a in api if s <= int(a["Start_Timestamp"]) <= e]
        names = []
        for a in launches:
            k = kern.get(a["Correlation_Id"])
            if k is not None:
                short = k["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1]
                names.append(f"{short} ({(int(k['End_Timestamp']) - int(k['Start_Timestamp'])) / 1e3:.2f} us)")
        inside_total += len(launches)
        print(f"{m['Function']:45s} host {(e - s) / 1e3:7.2f} us  launches {len(launches)}: {', '.join(names)}")
    print(f"\n{len(marks)} ranges, {inside_total} kernel launches inside them")


if __name__ == "__main__":
    main()
