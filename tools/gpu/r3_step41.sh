#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python benchmarks/bench_forward.py > gpurun_out/r3_bench_forward.jsonl 2>gpurun_out/r3_bench_forward.err || { tail -20 gpurun_out/r3_bench_forward.err; exit 1; }
cat gpurun_out/r3_bench_forward.jsonl
timeout -k 10 400 python -u -m pytest tests/test_native_update.py tests/test_kernels_gpu.py tests/test_state_arena.py tests/test_graphed_compute_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_s41_tests.log 2>&1 || { tail -30 gpurun_out/r3_s41_tests.log; exit 1; }
tail -1 gpurun_out/r3_s41_tests.log
