#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stream_kernels_gpu.py tests/test_bin_fused_finalize_gpu.py tests/test_sigmoid_cut_gpu.py -m gpu > gpurun_out/r5b2_tests.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert|passed|failed" gpurun_out/r5b2_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r5b2_tests.log
for m in 1 2; do
TM_AMD_BIN_VEC_BLOCKS_PER_CU=$m timeout -k 10 200 python3 benchmarks/bench_binary_stats.py > gpurun_out/r5b2_stats_$m.jsonl 2>&1 || { tail -5 gpurun_out/r5b2_stats_$m.jsonl; exit 1; }
echo "blocks/CU=$m"; grep '^{' gpurun_out/r5b2_stats_$m.jsonl | grep -i "multilabel\|Binary" | cut -c1-150
done
