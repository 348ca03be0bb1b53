#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_topk_gpu.py tests/test_sklearn_pinned_gpu.py tests/test_native_update.py tests/test_kernel_boundaries_gpu.py tests/test_determinism_gpu.py tests/test_wrappers.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_s43_tests.log 2>&1 || { tail -30 gpurun_out/r3_s43_tests.log; exit 1; }
tail -1 gpurun_out/r3_s43_tests.log
timeout -k 10 300 python benchmarks/bench_forward.py > gpurun_out/r3_bench_forward.jsonl 2>gpurun_out/r3_bench_forward.err || { tail -20 gpurun_out/r3_bench_forward.err; exit 1; }
cat gpurun_out/r3_bench_forward.jsonl
timeout -k 10 300 python benchmarks/forward_profile.py > gpurun_out/r3_forward_profile.txt 2>&1 || exit 1
grep " us " gpurun_out/r3_forward_profile.txt
