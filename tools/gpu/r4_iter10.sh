#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
T="tests/test_fused_compute_gpu.py tests/test_compute_groups.py tests/test_graphed_compute_gpu.py tests/test_collection_checks_gpu.py tests/test_regression.py"
timeout -k 10 300 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i10_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i10_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
for i in 1 2; do
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step 2>gpurun_out/r4i10_coll.err > gpurun_out/r4i10_collection_$i.json || { tail -20 gpurun_out/r4i10_coll.err; exit 1; }
cut -c1-250 gpurun_out/r4i10_collection_$i.json
done
timeout -k 10 200 python benchmarks/collection_phases.py --profile gpurun_out/r4i10_collection_profile.txt > gpurun_out/r4i10_collection_phases.json 2>gpurun_out/r4i10_phases.err || { tail -20 gpurun_out/r4i10_phases.err; exit 1; }
cat gpurun_out/r4i10_collection_phases.json
