#!/bin/bash
# Aggregation / exact-match tests and bench after the 16-byte load change.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_aggregation_gpu.py tests/test_exact_match_gpu.py tests/test_determinism_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/agg_gpu.log 2>&1 || { tail -40 gpurun_out/agg_gpu.log; exit 1; }
tail -1 gpurun_out/agg_gpu.log
timeout -k 10 300 python -u benchmarks/bench_aggregation.py > gpurun_out/bench_agg.jsonl 2> gpurun_out/bench_agg.err || { tail -20 gpurun_out/bench_agg.err; exit 1; }
cat gpurun_out/bench_agg.jsonl
