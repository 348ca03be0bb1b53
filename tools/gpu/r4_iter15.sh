#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_regression.py tests/test_fused_compute_gpu.py tests/test_precision_grad.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i15_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i15_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step 2>gpurun_out/r4i15_coll.err > gpurun_out/r4i15_collection.json || { tail -20 gpurun_out/r4i15_coll.err; exit 1; }
cut -c1-250 gpurun_out/r4i15_collection.json
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_coll -o p -- python3 $R/benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step --no-baseline > $R/gpurun_out/r4i15_coll.log 2>&1 || { tail -20 $R/gpurun_out/r4i15_coll.log; exit 1; }
cd $R && python3 tools/gpu/trace_summary.py gpurun_out/prof_coll --calls 111 > gpurun_out/r4i15_coll_trace.txt && grep -E "moments|total" gpurun_out/r4i15_coll_trace.txt | cut -c1-140 && rm -rf gpurun_out/prof_coll
timeout -k 10 300 python benchmarks/bench_map.py 2>gpurun_out/r4i15_map.err > gpurun_out/r4i15_bench_map.json || { tail -20 gpurun_out/r4i15_map.err; exit 1; }
cut -c1-250 gpurun_out/r4i15_bench_map.json
