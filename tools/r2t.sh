#!/bin/bash
# Aggregation / exact-match GPU step: their tests, the bench, and a rocprofv3 kernel-stats pass over the bench.
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH="$R"
timeout -k 10 300 python -u -m pytest tests/test_aggregation_gpu.py tests/test_exact_match_gpu.py tests/test_group_stats_gpu.py tests/test_determinism_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/agg_gpu.log 2>&1 || { tail -40 gpurun_out/agg_gpu.log; exit 1; }
tail -2 gpurun_out/agg_gpu.log
timeout -k 10 300 python -u benchmarks/bench_aggregation.py > gpurun_out/bench_agg.jsonl 2> gpurun_out/bench_agg.err || { tail -20 gpurun_out/bench_agg.err; exit 1; }
cat gpurun_out/bench_agg.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_agg -o p --output-format csv -- python3 $R/benchmarks/bench_aggregation.py > $R/gpurun_out/prof_agg.log 2>&1 || { tail -30 $R/gpurun_out/prof_agg.log; exit 1; }
cd $R && cp $(find gpurun_out/prof_agg -name "*kernel_stats.csv" | head -1) gpurun_out/agg_kernel_stats.csv && rm -rf gpurun_out/prof_agg
cut -d, -f1-4 gpurun_out/agg_kernel_stats.csv | head -20
