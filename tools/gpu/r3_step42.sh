#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python benchmarks/forward_profile.py > gpurun_out/r3_forward_profile.txt 2>&1 || { tail -20 gpurun_out/r3_forward_profile.txt; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/fwdprof -o f -- python3 $GRAFT_REPO_ROOT/benchmarks/forward_profile.py > /dev/null 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && cp $(find gpurun_out/fwdprof -name "*kernel_stats.csv" | head -1) gpurun_out/r3_forward_kernel_stats.csv && rm -rf gpurun_out/fwdprof
