#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
T="tests/test_detection.py tests/test_iou_module.py tests/test_fused_compute_gpu.py tests/test_compute_groups.py tests/test_graphed_compute_gpu.py"
timeout -k 10 300 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i9_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i9_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 300 python benchmarks/bench_map.py 2>gpurun_out/r4i9_map.err > gpurun_out/r4i9_bench_map.json || { tail -20 gpurun_out/r4i9_map.err; exit 1; }
cut -c1-300 gpurun_out/r4i9_bench_map.json
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step 2>gpurun_out/r4i9_coll.err > gpurun_out/r4i9_collection.json || { tail -20 gpurun_out/r4i9_coll.err; exit 1; }
cut -c1-300 gpurun_out/r4i9_collection.json
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 2>gpurun_out/r4i9_coll_u.err > gpurun_out/r4i9_collection_update.json || { tail -20 gpurun_out/r4i9_coll_u.err; exit 1; }
cut -c1-300 gpurun_out/r4i9_collection_update.json
timeout -k 10 200 python benchmarks/collection_phases.py --profile gpurun_out/r4i9_collection_profile.txt > gpurun_out/r4i9_collection_phases.json 2>gpurun_out/r4i9_phases.err || { tail -20 gpurun_out/r4i9_phases.err; exit 1; }
cat gpurun_out/r4i9_collection_phases.json
