#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_sklearn_pinned_gpu.py tests/test_kernel_boundaries_gpu.py tests/test_native_update.py tests/test_topk_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_s53_tests.log 2>&1 || { tail -30 gpurun_out/r3_s53_tests.log; exit 1; }
tail -1 gpurun_out/r3_s53_tests.log
timeout -k 10 300 python benchmarks/bench_binary_stats.py 2>/dev/null | tee gpurun_out/r3_bench_stats_updates.jsonl
