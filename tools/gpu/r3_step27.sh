#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u benchmarks/map_compute_cprofile.py > gpurun_out/r3_s27_cprof.txt 2>&1 || { tail -30 gpurun_out/r3_s27_cprof.txt; exit 1; }
timeout -k 10 300 python -u benchmarks/map_compute_cprofile.py --extended > gpurun_out/r3_s27_cprof_ext.txt 2>&1 || { tail -30 gpurun_out/r3_s27_cprof_ext.txt; exit 1; }
