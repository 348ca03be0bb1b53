#!/bin/bash
# Average device time of one kernel under a set of environment variants: for each "VAR=val ..." argument, run
#   rocprofv3 --kernel-trace --stats -- python3 <script>
# and print the variant with the matching kernel's calls / average / min / max (gpurun_out/<name>_sweep.jsonl).
#   bash tools/gpu/kstat_sweep.sh <name> <script> <kernel-substring> "<env variant>" ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
N=$1; S=$2; K=$3; shift 3
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  d=$R/gpurun_out/${N}_sw
  rm -rf $d
  ( cd /tmp && export $v && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o p --output-format csv -- python3 $R/$S > $R/gpurun_out/${N}_sw.log 2>&1 ) || { echo "variant $v failed"; tail -20 $R/gpurun_out/${N}_sw.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$K" "$v" >> $R/gpurun_out/${N}_sweep.jsonl <<'PY'
import csv, json, sys
f, k, v = sys.argv[1:4]
rows = [r for r in csv.DictReader(open(f)) if k in r["Name"]]
out = {"variant": v}
for r in rows:
    out[r["Name"][:60]] = {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
                           "min_us": round(float(r["MinNs"]) / 1e3, 2), "max_us": round(float(r["MaxNs"]) / 1e3, 2)}
print(json.dumps(out))
PY
  tail -1 $R/gpurun_out/${N}_sweep.jsonl
  rm -rf $d
done
