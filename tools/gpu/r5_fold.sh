#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
TM_AMD_BIN_FOLD_MIN_BLOCKS=64 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stream_kernels_gpu.py tests/test_bin_fused_finalize_gpu.py -m gpu > gpurun_out/r5fo_tests.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert|passed|failed" gpurun_out/r5fo_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r5fo_tests.log
for m in 32 0 32 0 32; do
TM_AMD_BIN_FOLD_MIN_BLOCKS=$m timeout -k 10 200 python3 benchmarks/bench_binary_stats.py > gpurun_out/r5fo_$m.jsonl 2>&1 || { tail -5 gpurun_out/r5fo_$m.jsonl; exit 1; }
echo "min_blocks=$m $(grep '^{' gpurun_out/r5fo_$m.jsonl | grep -i multilabel | cut -c1-100 | tr '\n' ' ')"
done
