#!/bin/bash
# Round-4 iteration call: diagnostics of the native-forward decline and the fp64 interp mismatch, the GPU tests of
# this round's fixes, the benches the first call did not reach, and a kernel trace of the stat-score updates.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python tools/gpu/diag_forward.py > gpurun_out/r4i_diag_forward.log 2>&1 || { tail -30 gpurun_out/r4i_diag_forward.log; exit 1; }
timeout -k 10 60 python tools/gpu/diag_interp.py > gpurun_out/r4i_diag_interp.log 2>&1 || { tail -30 gpurun_out/r4i_diag_interp.log; exit 1; }
cat gpurun_out/r4i_diag_interp.log | head -20
T="tests/test_fused_compute_gpu.py tests/test_gemm_big_gpu.py tests/test_macro_curves.py tests/test_torchscript.py tests/test_engine_gpu.py tests/test_ddp.py tests/test_oneshot_gpu.py tests/test_compute_groups.py tests/test_graphed_compute_gpu.py tests/test_collection_checks_gpu.py"
timeout -k 10 500 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i_pytest.log | tail -30
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step 2>gpurun_out/r4i_collection.err > gpurun_out/r4i_collection.json || { tail -20 gpurun_out/r4i_collection.err; exit 1; }
cut -c1-600 gpurun_out/r4i_collection.json
timeout -k 10 300 python benchmarks/bench_map.py 2>gpurun_out/r4i_map.err > gpurun_out/r4i_bench_map.json || { tail -20 gpurun_out/r4i_map.err; exit 1; }
cut -c1-400 gpurun_out/r4i_bench_map.json
timeout -k 10 300 python benchmarks/bench_gemm.py 2>gpurun_out/r4i_gemm.err > gpurun_out/r4i_bench_gemm.jsonl || { tail -20 gpurun_out/r4i_gemm.err; exit 1; }
cut -c1-300 gpurun_out/r4i_bench_gemm.jsonl
timeout -k 10 120 python benchmarks/bench_word_read.py 2>/dev/null > gpurun_out/r4i_word_read.jsonl || exit 1
cat gpurun_out/r4i_word_read.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o p -- python3 $R/benchmarks/bench_binary_stats.py > $R/gpurun_out/r4i_prof_stats.log 2>&1 || { tail -20 $R/gpurun_out/r4i_prof_stats.log; exit 1; }
cd $R && cp $(find gpurun_out/prof_stats -name "*kernel_stats.csv" | head -1) gpurun_out/r4i_stats_kernel_stats.csv && rm -rf gpurun_out/prof_stats
cut -d, -f1-8 gpurun_out/r4i_stats_kernel_stats.csv | cut -c1-220 | head -16
