#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python benchmarks/forward_phases.py 2>/dev/null | tee gpurun_out/r3_forward_phases.jsonl
