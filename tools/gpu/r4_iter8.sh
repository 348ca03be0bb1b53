#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
T="tests/test_stream_kernels_gpu.py tests/test_kernel_boundaries_gpu.py tests/test_kernels_gpu.py tests/test_classification_stats.py tests/test_native_forward_gpu.py"
timeout -k 10 300 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i8_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i8_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 120 python benchmarks/bench_fewbins.py > gpurun_out/r4i8_fewbins.jsonl 2>gpurun_out/r4i8_fewbins.err || { tail -20 gpurun_out/r4i8_fewbins.err; exit 1; }
tr -d '{}"' < gpurun_out/r4i8_fewbins.jsonl | paste -sd';' | fold -w 4000
timeout -k 10 200 python benchmarks/bench_binary_stats.py > gpurun_out/r4i8_stats.jsonl 2>/dev/null || exit 1
tail -2 gpurun_out/r4i8_stats.jsonl
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_coll -o p -- python3 $R/benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step --no-baseline > $R/gpurun_out/r4i8_coll.log 2>&1 || { tail -20 $R/gpurun_out/r4i8_coll.log; exit 1; }
cd $R && python3 tools/gpu/trace_summary.py gpurun_out/prof_coll --calls 111 > gpurun_out/r4i8_coll_trace.txt && head -8 gpurun_out/r4i8_coll_trace.txt | cut -c1-140 && tail -1 gpurun_out/r4i8_coll_trace.txt && rm -rf gpurun_out/prof_coll
