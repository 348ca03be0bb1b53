#!/bin/bash
# Few-class multiclass update (mc_fewbins_tile_kernel): GPU tests of the tiled kernel, then bench_mc_small.py under
# env variants (group hand-off vs fold launch, rows per tile, blocks per CU), then a kernel-stats pass of the default.
#   bash tools/gpu/mc_small.sh <name> "<env variant>" ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
N=$1; shift
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_stream_kernels_gpu.py tests/test_moments_handoff_gpu.py -m gpu -x -q \
  --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${N}_tests.log 2>&1 || { tail -30 gpurun_out/${N}_tests.log; exit 1; }
tail -3 gpurun_out/${N}_tests.log
for v in "$@"; do
  ( export $v && timeout -k 10 120 python3 -u benchmarks/bench_mc_small.py >> gpurun_out/${N}_bench.jsonl 2>> gpurun_out/${N}_bench.err ) || { echo "variant $v failed"; tail -20 gpurun_out/${N}_bench.err; exit 1; }
done
cat gpurun_out/${N}_bench.jsonl
d=$R/gpurun_out/${N}_prof
( cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o p --output-format csv -- python3 $R/benchmarks/bench_mc_small.py > $R/gpurun_out/${N}_prof.log 2>&1 ) || { tail -20 $R/gpurun_out/${N}_prof.log; exit 1; }
f=$(find $d -name "*kernel_stats.csv" | head -1)
cp $f gpurun_out/${N}_kernel_stats.csv
head -8 gpurun_out/${N}_kernel_stats.csv
rm -rf $d
