#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fused_update_gpu.py tests/test_fused_compute_gpu.py tests/test_calibration_cache_gpu.py tests/test_classification_extras.py -m gpu > gpurun_out/r5c_tests.log 2>&1 || { tail -30 gpurun_out/r5c_tests.log; exit 1; }
tail -1 gpurun_out/r5c_tests.log
for i in 1 2; do
timeout -k 10 300 python3 benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 > gpurun_out/r5c_sync_$i.json 2>&1 || { tail -5 gpurun_out/r5c_sync_$i.json; exit 1; }
tail -1 gpurun_out/r5c_sync_$i.json | cut -c1-250; tail -1 gpurun_out/r5c_sync_$i.json | grep -o '"phases_ms_per_step_max_over_ranks": {[^}]*}'
done
timeout -k 10 300 python3 benchmarks/bench_collection.py --steps 200 --warmup 20 > gpurun_out/r5c_upd.json 2>&1 || { tail -5 gpurun_out/r5c_upd.json; exit 1; }
tail -1 gpurun_out/r5c_upd.json | cut -c1-250
