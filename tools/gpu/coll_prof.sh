#!/bin/bash
# Config #5 (bench_collection.py, eager, compute every step): phases JSON, an ours-only kernel trace and cProfile of
# the classification / regression compute path.  Logs under gpurun_out/<name>_*.
#   bash tools/gpu/coll_prof.sh <name>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
N=${1:-coll}
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python benchmarks/bench_collection.py --steps 200 --warmup 20 --sync-every-step --no-baseline > gpurun_out/${N}_phases.log 2>&1 || { tail -20 gpurun_out/${N}_phases.log; exit 1; }
grep '^{' gpurun_out/${N}_phases.log | tail -1 | cut -c1-900
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${N}_prof -o p --output-format csv -- python3 $R/benchmarks/bench_collection.py --steps 200 --warmup 20 --sync-every-step --no-baseline > $R/gpurun_out/${N}_prof.log 2>&1 || { tail -20 $R/gpurun_out/${N}_prof.log; exit 1; }
cd $R && f=$(find gpurun_out/${N}_prof -name "*kernel_stats.csv" | head -1) && cp $f gpurun_out/${N}_kernel_stats.csv && cut -d, -f1-5 gpurun_out/${N}_kernel_stats.csv | head -20
find gpurun_out/${N}_prof -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/${N}_kernel_trace.csv
rm -rf gpurun_out/${N}_prof
for w in cls reg; do
  timeout -k 10 120 python benchmarks/compute_cprofile.py --which $w > gpurun_out/${N}_cprof_$w.log 2>&1 || { tail -20 gpurun_out/${N}_cprof_$w.log; exit 1; }
done
head -45 gpurun_out/${N}_cprof_cls.log
