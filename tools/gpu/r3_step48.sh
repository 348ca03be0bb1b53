#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python benchmarks/bench_binary_stats.py 2>/dev/null | tee gpurun_out/r3_bench_binary_stats.jsonl
