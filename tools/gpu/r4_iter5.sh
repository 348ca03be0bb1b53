#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
T="tests/test_stream_kernels_gpu.py tests/test_kernel_boundaries_gpu.py tests/test_kernels_gpu.py tests/test_native_forward_gpu.py tests/test_classification_stats.py tests/test_sklearn_pinned_gpu.py"
timeout -k 10 300 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i5_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i5_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
for tile in 2 4 8; do
  TM_AMD_FEWBINS_TILE=$tile timeout -k 10 120 python benchmarks/bench_fewbins.py >> gpurun_out/r4i5_fewbins.jsonl 2>gpurun_out/r4i5_fewbins.err || { tail -20 gpurun_out/r4i5_fewbins.err; exit 1; }
done
tr -d '{}"' < gpurun_out/r4i5_fewbins.jsonl | paste -sd';' | fold -w 4000
timeout -k 10 200 python benchmarks/bench_binary_stats.py > gpurun_out/r4i5_stats.jsonl 2>/dev/null || exit 1
cat gpurun_out/r4i5_stats.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4i5_bench20_$i.log 2>&1 || { tail -30 gpurun_out/r4i5_bench20_$i.log; exit 1; }
  grep '^{' gpurun_out/r4i5_bench20_$i.log | cut -c1-200
done
