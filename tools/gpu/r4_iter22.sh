#!/bin/bash
# binary / multilabel kernels with per-block partials + partials_fold_kernel: tests, stats-update bench, kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stream_kernels_gpu.py tests/test_kernels_gpu.py tests/test_sklearn_pinned_gpu.py tests/test_determinism_gpu.py tests/test_native_forward_gpu.py tests/test_kernel_boundaries_gpu.py tests/test_fused_compute_gpu.py tests/test_engine_gpu.py -m gpu > gpurun_out/r4i22_tests.log 2>&1 || { tail -30 gpurun_out/r4i22_tests.log; exit 1; }
tail -1 gpurun_out/r4i22_tests.log
timeout -k 10 200 python benchmarks/bench_binary_stats.py > gpurun_out/r4i22_stats.jsonl 2>&1 || { tail -5 gpurun_out/r4i22_stats.jsonl; exit 1; }
grep case gpurun_out/r4i22_stats.jsonl
cd /tmp
d=$R/gpurun_out/r4i22_trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o p -- python3 $R/benchmarks/bench_binary_stats.py > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 $R/tools/gpu/trace_summary.py $d --match _kernel | cut -c1-150 | grep -v "^$" | head -16
