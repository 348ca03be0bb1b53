#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_regression.py tests/test_fused_compute_gpu.py tests/test_compute_groups.py tests/test_precision_grad.py tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i14_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i14_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step 2>gpurun_out/r4i14_coll.err > gpurun_out/r4i14_collection.json || { tail -20 gpurun_out/r4i14_coll.err; exit 1; }
cut -c1-250 gpurun_out/r4i14_collection.json
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_coll -o p -- python3 $R/benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step --no-baseline > $R/gpurun_out/r4i14_coll.log 2>&1 || { tail -20 $R/gpurun_out/r4i14_coll.log; exit 1; }
cd $R && python3 tools/gpu/trace_summary.py gpurun_out/prof_coll --calls 111 > gpurun_out/r4i14_coll_trace.txt && head -12 gpurun_out/r4i14_coll_trace.txt | cut -c1-140 && tail -1 gpurun_out/r4i14_coll_trace.txt && rm -rf gpurun_out/prof_coll
timeout -k 10 120 python benchmarks/map_update_profile.py > gpurun_out/r4i14_map_profile.txt 2>&1 || { tail -20 gpurun_out/r4i14_map_profile.txt; exit 1; }
head -40 gpurun_out/r4i14_map_profile.txt | cut -c1-150
timeout -k 10 200 python -u -m pytest tests/test_native_forward_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i14_fwd_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i14_fwd_pytest.log | head -5
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 300 python benchmarks/bench_forward.py 2>gpurun_out/r4i14_forward.err > gpurun_out/r4i14_bench_forward.jsonl || { tail -20 gpurun_out/r4i14_forward.err; exit 1; }
cut -c1-230 gpurun_out/r4i14_bench_forward.jsonl
