#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_s33_fid -o fid -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_fid.py --no-baseline > $GRAFT_REPO_ROOT/gpurun_out/r3_s33.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_s33.log; exit 1; }
tail -2 $GRAFT_REPO_ROOT/gpurun_out/r3_s33.log
