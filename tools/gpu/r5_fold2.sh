#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests -m gpu > gpurun_out/r5fo2_tests.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert|passed|failed" gpurun_out/r5fo2_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r5fo2_tests.log
timeout -k 10 200 python3 benchmarks/bench_binary_stats.py > gpurun_out/r5fo2_stats.jsonl 2>&1 || { tail -5 gpurun_out/r5fo2_stats.jsonl; exit 1; }
grep '^{' gpurun_out/r5fo2_stats.jsonl | cut -c1-120
