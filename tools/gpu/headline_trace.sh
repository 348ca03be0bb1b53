#!/bin/bash
# Headline (bench.py) ours-only kernel statistics over a 200-step run: per-kernel calls / avg / min / max.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
N=${1:-hl}
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${N}_prof -o p --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-baseline > $R/gpurun_out/${N}_prof.log 2>&1 || { tail -20 $R/gpurun_out/${N}_prof.log; exit 1; }
cd $R && f=$(find gpurun_out/${N}_prof -name "*kernel_stats.csv" | head -1) && cp $f gpurun_out/${N}_kernel_stats.csv
find gpurun_out/${N}_prof -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/${N}_kernel_trace.csv
rm -rf gpurun_out/${N}_prof
cut -d, -f1-7 gpurun_out/${N}_kernel_stats.csv | cut -c1-200 | head -8
grep '^{' gpurun_out/${N}_prof.log | tail -1 | cut -c1-300
