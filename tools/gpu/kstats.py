"""Print name / calls / average / min / max (us) of the kernels in a rocprofv3 --stats output dir whose name matches."""
import csv
import glob
import sys

d = sys.argv[1]
pats = sys.argv[2:] or [""]
f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(p in n for p in pats):
        short = n.replace("(anonymous namespace)::", "").split("(")[0][:70]
        print(f"{short:72s} calls={r['Calls']:>6s} avg={float(r['AverageNs'])/1e3:8.2f}us "
              f"min={float(r['MinNs'])/1e3:7.2f} max={float(r['MaxNs'])/1e3:7.2f}")
