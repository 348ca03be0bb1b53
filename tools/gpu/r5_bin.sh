#!/bin/bash
# branch-free binary counters: full GPU suite, stat-score update bench, its ours-only kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5b_pytest_gpu.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|passed|failed" gpurun_out/r5b_pytest_gpu.log | tail -30; exit 1; }
tail -1 gpurun_out/r5b_pytest_gpu.log
timeout -k 10 200 python3 benchmarks/bench_binary_stats.py > gpurun_out/r5b_stats.jsonl 2>&1 || { tail -5 gpurun_out/r5b_stats.jsonl; exit 1; }
grep '^{' gpurun_out/r5b_stats.jsonl | cut -c1-150
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ps -o p -- python3 $R/benchmarks/bench_binary_stats.py > $R/gpurun_out/ps.log 2>&1 || { tail -5 $R/gpurun_out/ps.log; exit 1; }
cd $R && cp $(find gpurun_out/ps -name "*kernel_stats.csv" | head -1) gpurun_out/r5b_stats_kernel_stats.csv && python3 tools/gpu/kstats.py gpurun_out/ps bin_ fewbins argmax finalize | head -14; rm -rf gpurun_out/ps
