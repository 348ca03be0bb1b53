#!/bin/bash
# topk kernel tests + stat-scores suites on the GPU, then the misc kernel bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_topk_gpu.py tests/test_classification_stats.py -m gpu > gpurun_out/r2q.log 2>&1
rc=$?; tail -5 gpurun_out/r2q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/bench_misc_kernels.py > gpurun_out/r2r_misc.jsonl 2> gpurun_out/r2r_misc.err
rc=$?; cat gpurun_out/r2r_misc.jsonl; exit $rc
