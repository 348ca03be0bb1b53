#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u benchmarks/collection_compute_eager.py > gpurun_out/r3_s15_coll_eager.json 2>&1 || { tail -30 gpurun_out/r3_s15_coll_eager.json; exit 1; }
cat gpurun_out/r3_s15_coll_eager.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_s15_prof -o coll -- python3 $GRAFT_REPO_ROOT/benchmarks/collection_compute_eager.py --loop 100 > $GRAFT_REPO_ROOT/gpurun_out/r3_s15_prof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/r3_s15_prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r3_s15_prof -name "*stats*"
