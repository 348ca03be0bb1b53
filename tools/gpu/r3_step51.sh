#!/bin/bash
# kernel trace of the forward probe after the stats fixes (accuracy stats workspace through the order-key kernel)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/fwdprof -o f -- python3 $GRAFT_REPO_ROOT/benchmarks/forward_profile.py > /dev/null 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && cp $(find gpurun_out/fwdprof -name "*kernel_stats.csv" | head -1) gpurun_out/r3_forward_kernel_stats_after.csv && rm -rf gpurun_out/fwdprof
cut -d, -f1-4 gpurun_out/r3_forward_kernel_stats_after.csv | cut -c1-150 | head -8
