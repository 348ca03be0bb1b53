#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
T="tests/test_stream_kernels_gpu.py tests/test_kernel_boundaries_gpu.py tests/test_kernels_gpu.py tests/test_classification_stats.py tests/test_native_forward_gpu.py tests/test_native_update.py tests/test_sklearn_pinned_gpu.py tests/test_engine_gpu.py"
timeout -k 10 300 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i12_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i12_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 120 python benchmarks/bench_fewbins.py > gpurun_out/r4i12_fewbins.jsonl 2>gpurun_out/r4i12_fewbins.err || { tail -20 gpurun_out/r4i12_fewbins.err; exit 1; }
tr -d '{}"' < gpurun_out/r4i12_fewbins.jsonl | paste -sd';' | fold -w 4000
timeout -k 10 200 python benchmarks/bench_binary_stats.py > gpurun_out/r4i12_stats.jsonl 2>/dev/null || exit 1
cat gpurun_out/r4i12_stats.jsonl
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step 2>gpurun_out/r4i12_coll.err > gpurun_out/r4i12_collection.json || { tail -20 gpurun_out/r4i12_coll.err; exit 1; }
cut -c1-250 gpurun_out/r4i12_collection.json
