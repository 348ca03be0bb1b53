#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 200 python benchmarks/collection_host_breakdown.py > gpurun_out/r4i16_breakdown.json 2>gpurun_out/r4i16_bd.err || { tail -20 gpurun_out/r4i16_bd.err; exit 1; }
cat gpurun_out/r4i16_breakdown.json
