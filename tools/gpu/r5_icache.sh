#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ic -o p -- $R/benchmarks/native/icache_probe > $R/gpurun_out/ic.log 2>&1 || { tail -5 $R/gpurun_out/ic.log; exit 1; }
cd $R && python3 tools/gpu/kstats.py gpurun_out/ic "" | tee gpurun_out/r5_icache.txt; rm -rf gpurun_out/ic
