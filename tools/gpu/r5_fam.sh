#!/bin/bash
# Round 5: fused collection update (family.hip) + single-block moments: GPU tests, config #5 bench, kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fused_update_gpu.py tests/test_fused_compute_gpu.py tests/test_stream_kernels_gpu.py tests/test_native_update.py tests/test_native_forward_gpu.py tests/test_kernels_gpu.py tests/test_sklearn_pinned_gpu.py tests/test_torchscript.py tests/test_state_arena.py tests/test_exact_match_gpu.py tests/test_curve_views.py tests/test_classification_curves.py tests/test_sigmoid_cut_gpu.py tests/test_bin_fused_finalize_gpu.py tests/test_clustering_gpu.py tests/test_classification_stats.py -m gpu > gpurun_out/r5fam_tests.log 2>&1 || { tail -40 gpurun_out/r5fam_tests.log; exit 1; }
tail -2 gpurun_out/r5fam_tests.log
timeout -k 10 300 python3 benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 > gpurun_out/r5fam_coll_sync.json 2>&1 || { tail -5 gpurun_out/r5fam_coll_sync.json; exit 1; }
tail -1 gpurun_out/r5fam_coll_sync.json | cut -c1-700
timeout -k 10 300 python3 benchmarks/bench_collection.py --steps 200 --warmup 20 > gpurun_out/r5fam_coll_upd.json 2>&1 || { tail -5 gpurun_out/r5fam_coll_upd.json; exit 1; }
tail -1 gpurun_out/r5fam_coll_upd.json | cut -c1-700
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5fam_prof -o p -- python3 $R/benchmarks/bench_collection.py --sync-every-step --steps 100 --warmup 10 --no-baseline > $R/gpurun_out/r5fam_prof.log 2>&1 || { tail -20 $R/gpurun_out/r5fam_prof.log; exit 1; }
cd $R && python3 tools/gpu/trace_summary.py gpurun_out/r5fam_prof --calls 110 > gpurun_out/r5fam_trace_summary.txt; head -30 gpurun_out/r5fam_trace_summary.txt; tail -1 gpurun_out/r5fam_trace_summary.txt
timeout -k 10 200 python3 benchmarks/bench_binary_stats.py > gpurun_out/r5fam_stats.jsonl 2>&1 || { tail -5 gpurun_out/r5fam_stats.jsonl; exit 1; }
grep case gpurun_out/r5fam_stats.jsonl
