#!/bin/bash
# Config #3 (bench_map.py): the bench line, a kernel-trace of compute() (map_compute_cprofile.py) and its cProfile.
#   bash tools/gpu/map_prof.sh <name>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
N=${1:-map}
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python benchmarks/bench_map.py > gpurun_out/${N}_bench.log 2>&1 || { tail -20 gpurun_out/${N}_bench.log; exit 1; }
grep '^{' gpurun_out/${N}_bench.log | tail -1 | cut -c1-400
timeout -k 10 300 python benchmarks/map_compute_cprofile.py > gpurun_out/${N}_cprof.log 2>&1 || { tail -20 gpurun_out/${N}_cprof.log; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${N}_prof -o p --output-format csv -- python3 $R/benchmarks/map_compute_cprofile.py > $R/gpurun_out/${N}_prof.log 2>&1 || { tail -20 $R/gpurun_out/${N}_prof.log; exit 1; }
cd $R && f=$(find gpurun_out/${N}_prof -name "*kernel_stats.csv" | head -1) && cp $f gpurun_out/${N}_kernel_stats.csv
rm -rf gpurun_out/${N}_prof
