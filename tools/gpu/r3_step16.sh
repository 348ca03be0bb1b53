#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u benchmarks/compute_cprofile.py > gpurun_out/r3_s16_cprofile.txt 2>&1 || { tail -30 gpurun_out/r3_s16_cprofile.txt; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_s16_prof -o coll -- python3 $GRAFT_REPO_ROOT/benchmarks/collection_compute_eager.py --loop 100 > $GRAFT_REPO_ROOT/gpurun_out/r3_s16_prof.txt 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/r3_s16_prof.txt; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r3_s16_prof -name "*stats*"
