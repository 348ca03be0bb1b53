#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 benchmarks/bench_forward.py > gpurun_out/r5fwd.jsonl 2>&1 || { tail -5 gpurun_out/r5fwd.jsonl; exit 1; }
grep '^{' gpurun_out/r5fwd.jsonl | cut -c1-260
timeout -k 10 300 python3 benchmarks/bench_clustering.py > gpurun_out/r5clu.jsonl 2>&1 || { tail -5 gpurun_out/r5clu.jsonl; exit 1; }
grep '^{' gpurun_out/r5clu.jsonl | cut -c1-200
