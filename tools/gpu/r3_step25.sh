#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u benchmarks/map_compute_phases.py > gpurun_out/r3_s25_map_phases.json 2>&1 || { tail -30 gpurun_out/r3_s25_map_phases.json; exit 1; }
cat gpurun_out/r3_s25_map_phases.json
