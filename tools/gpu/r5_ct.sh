#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fused_compute_gpu.py tests/test_graphed_compute_gpu.py tests/test_fused_update_gpu.py tests/test_collection_checks_gpu.py tests/test_fused_misc_gpu.py -m gpu > gpurun_out/r5ct_tests.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert|passed|failed" gpurun_out/r5ct_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r5ct_tests.log
for i in 1 2; do
timeout -k 10 300 python3 benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 > gpurun_out/r5ct_sync_$i.json 2>&1 || { tail -5 gpurun_out/r5ct_sync_$i.json; exit 1; }
tail -1 gpurun_out/r5ct_sync_$i.json | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"phases_ms_per_step_max_over_ranks": {[^}]*}' | tr '\n' ' '; echo
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pc -o p -- python3 $R/benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 --no-baseline > $R/gpurun_out/pc.log 2>&1 || { tail -5 $R/gpurun_out/pc.log; exit 1; }
cd $R && cp $(find gpurun_out/pc -name "*kernel_stats.csv" | head -1) gpurun_out/r5ct_collection_sync_kernel_stats.csv && python3 tools/gpu/kstats.py gpurun_out/pc tm_amd | head -8; rm -rf gpurun_out/pc
