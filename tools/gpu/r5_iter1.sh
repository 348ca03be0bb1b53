#!/bin/bash
# Round 5 iteration: stat kernels (fused fold+finalize block shape), moments probe, config #5 with AUROC/AP fused.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fused_update_gpu.py tests/test_bin_fused_finalize_gpu.py tests/test_stream_kernels_gpu.py tests/test_kernels_gpu.py tests/test_fused_compute_gpu.py -m gpu > gpurun_out/r5i1_tests.log 2>&1 || { tail -40 gpurun_out/r5i1_tests.log; exit 1; }
tail -1 gpurun_out/r5i1_tests.log
timeout -k 10 200 python3 benchmarks/bench_binary_stats.py > gpurun_out/r5i1_stats.jsonl 2>&1 || { tail -5 gpurun_out/r5i1_stats.jsonl; exit 1; }
grep case gpurun_out/r5i1_stats.jsonl
timeout -k 10 200 python3 benchmarks/moments_probe.py > gpurun_out/r5i1_moments.jsonl 2>&1 || { tail -5 gpurun_out/r5i1_moments.jsonl; exit 1; }
grep '"n"' gpurun_out/r5i1_moments.jsonl
timeout -k 10 300 python3 benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 > gpurun_out/r5i1_coll_sync.json 2>&1 || { tail -5 gpurun_out/r5i1_coll_sync.json; exit 1; }
tail -1 gpurun_out/r5i1_coll_sync.json | cut -c1-900
timeout -k 10 300 python3 benchmarks/bench_collection.py --steps 200 --warmup 20 > gpurun_out/r5i1_coll_upd.json 2>&1 || { tail -5 gpurun_out/r5i1_coll_upd.json; exit 1; }
tail -1 gpurun_out/r5i1_coll_upd.json | cut -c1-500
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5i1_prof -o p -- python3 $R/benchmarks/bench_collection.py --sync-every-step --steps 100 --warmup 10 --no-baseline > $R/gpurun_out/r5i1_prof.log 2>&1 || { tail -20 $R/gpurun_out/r5i1_prof.log; exit 1; }
cd $R && python3 tools/gpu/trace_summary.py gpurun_out/r5i1_prof --calls 110 > gpurun_out/r5i1_trace_summary.txt; head -16 gpurun_out/r5i1_trace_summary.txt; tail -1 gpurun_out/r5i1_trace_summary.txt; rm -rf gpurun_out/r5i1_prof
