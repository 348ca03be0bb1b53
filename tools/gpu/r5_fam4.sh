#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fused_update_gpu.py tests/test_calibration_cache_gpu.py tests/test_stream_kernels_gpu.py tests/test_bin_fused_finalize_gpu.py tests/test_sigmoid_cut_gpu.py -m gpu > gpurun_out/r5f4_tests.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert|passed|failed" gpurun_out/r5f4_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r5f4_tests.log
for m in 1 2; do
TM_AMD_BIN_VEC_BLOCKS_PER_CU=$m timeout -k 10 200 python3 benchmarks/bench_binary_stats.py > gpurun_out/r5f4_stats_$m.jsonl 2>&1 || { tail -5 gpurun_out/r5f4_stats_$m.jsonl; exit 1; }
echo "blocks/CU=$m"; grep '^{' gpurun_out/r5f4_stats_$m.jsonl | grep -i "multilabel\|Binary" | cut -c1-150
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pc -o p -- python3 $R/benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 --no-baseline > $R/gpurun_out/pc.log 2>&1 || { tail -5 $R/gpurun_out/pc.log; exit 1; }
cd $R && cp $(find gpurun_out/pc -name "*kernel_stats.csv" | head -1) gpurun_out/r5f4_collection_sync_kernel_stats.csv && python3 tools/gpu/kstats.py gpurun_out/pc tm_amd | head -10; rm -rf gpurun_out/pc
