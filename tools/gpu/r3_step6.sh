#!/bin/bash
# kernel trace of the first-region probe: per-dispatch durations and gaps of the update kernel, region by region
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_fr -o fr -- python3 $R/benchmarks/first_region_probe.py plain > $R/gpurun_out/r3_fr_prof.log 2>&1 || { tail -20 $R/gpurun_out/r3_fr_prof.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_fr -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if "mc_argmax" in r["Kernel_Name"]]
print("update kernels:", len(ks))
prev_end = None
out = []
for i, r in enumerate(ks):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end else 0
    out.append((i, round((e - s) / 1e3, 2), round(gap, 2)))
    prev_end = e
for x in out: print(x)
PY
rm -rf gpurun_out/prof_fr
