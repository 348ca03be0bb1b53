#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pairwise_precision_gpu.py tests/test_gemm_kernels.py tests/test_pairwise.py -m gpu > gpurun_out/r3_s14_tests.log 2>&1 || { tail -40 gpurun_out/r3_s14_tests.log; exit 1; }
tail -3 gpurun_out/r3_s14_tests.log
timeout -k 10 300 python -u benchmarks/bench_pairwise.py > gpurun_out/r3_s14_pairwise.jsonl 2>&1 || { tail -30 gpurun_out/r3_s14_pairwise.jsonl; exit 1; }
cat gpurun_out/r3_s14_pairwise.jsonl
