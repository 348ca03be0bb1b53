#!/bin/bash
# small-grid atomic flush vs fold: tests, stats bench, config #5 collection
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stream_kernels_gpu.py tests/test_kernels_gpu.py tests/test_sklearn_pinned_gpu.py tests/test_determinism_gpu.py tests/test_native_forward_gpu.py tests/test_kernel_boundaries_gpu.py tests/test_fused_compute_gpu.py -m gpu > gpurun_out/r4i23_tests.log 2>&1 || { tail -30 gpurun_out/r4i23_tests.log; exit 1; }
tail -1 gpurun_out/r4i23_tests.log
timeout -k 10 200 python benchmarks/bench_binary_stats.py > gpurun_out/r4i23_stats.jsonl 2>&1 || { tail -5 gpurun_out/r4i23_stats.jsonl; exit 1; }
grep case gpurun_out/r4i23_stats.jsonl
timeout -k 10 300 python benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 > gpurun_out/r4i23_coll.json 2>&1 || { tail -5 gpurun_out/r4i23_coll.json; exit 1; }
tail -1 gpurun_out/r4i23_coll.json | cut -c1-400
timeout -k 10 200 python benchmarks/collection_host_breakdown.py > gpurun_out/r4i23_bd.json 2>&1 || { tail -5 gpurun_out/r4i23_bd.json; exit 1; }
tail -1 gpurun_out/r4i23_bd.json
