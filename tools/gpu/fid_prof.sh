#!/bin/bash
# Config #4 (FID, 50k x 2048): fp64 GEMM throughput (bench_dgemm.py), the FID bench line, and an ours-only kernel trace.
#   bash tools/gpu/fid_prof.sh <name> [skip_bench]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
N=${1:-fid}
R=$GRAFT_REPO_ROOT
timeout -k 10 240 python benchmarks/bench_dgemm.py > gpurun_out/${N}_dgemm.jsonl 2>&1 || { tail -20 gpurun_out/${N}_dgemm.jsonl; exit 1; }
grep '^{' gpurun_out/${N}_dgemm.jsonl | cut -c1-200
if [ -z "$2" ]; then
  timeout -k 10 300 python benchmarks/bench_fid.py > gpurun_out/${N}_bench.log 2>&1 || { tail -20 gpurun_out/${N}_bench.log; exit 1; }
  grep '^{' gpurun_out/${N}_bench.log | tail -1 | cut -c1-900
fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${N}_prof -o p --output-format csv -- python3 $R/benchmarks/bench_fid.py --ours-only > $R/gpurun_out/${N}_prof.log 2>&1 || { tail -20 $R/gpurun_out/${N}_prof.log; exit 1; }
cd $R && f=$(find gpurun_out/${N}_prof -name "*kernel_stats.csv" | head -1) && cp $f gpurun_out/${N}_kernel_stats.csv
rm -rf gpurun_out/${N}_prof
cut -d, -f1-4 gpurun_out/${N}_kernel_stats.csv | cut -c1-160 | head -12
