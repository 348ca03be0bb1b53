#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python benchmarks/compute_cprofile.py > gpurun_out/r3_compute_cprofile.txt 2>&1 || { tail -20 gpurun_out/r3_compute_cprofile.txt; exit 1; }
head -5 gpurun_out/r3_compute_cprofile.txt
