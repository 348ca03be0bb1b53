#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_fused_compute_gpu.py tests/test_compute_groups.py tests/test_collection_checks_gpu.py tests/test_graphed_compute_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i17_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i17_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 200 python benchmarks/collection_host_breakdown.py > gpurun_out/r4i17_breakdown.json 2>gpurun_out/r4i17_bd.err || { tail -20 gpurun_out/r4i17_bd.err; exit 1; }
cat gpurun_out/r4i17_breakdown.json
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step 2>gpurun_out/r4i17_coll.err > gpurun_out/r4i17_collection.json || { tail -20 gpurun_out/r4i17_coll.err; exit 1; }
cut -c1-250 gpurun_out/r4i17_collection.json
