#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r3_s30_counters.txt 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_s30_counters.txt; exit 1; }
grep -c . $GRAFT_REPO_ROOT/gpurun_out/r3_s30_counters.txt
