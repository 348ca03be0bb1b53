#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_h16_gpu.py tests/test_pairwise.py -m gpu > gpurun_out/r5g6_tests.log 2>&1 || { tail -30 gpurun_out/r5g6_tests.log; exit 1; }
tail -1 gpurun_out/r5g6_tests.log
timeout -k 10 200 python3 benchmarks/bench_gemm16.py > gpurun_out/r5g6_bench.jsonl 2>&1 || { tail -5 gpurun_out/r5g6_bench.jsonl; exit 1; }
grep -h shape gpurun_out/r5g6_bench.jsonl | grep bfloat16 | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(' ', d['shape'], 'store', d['store_ms'], 'cos', d['pairwise_cosine_ms'], 'cosgemm', d['cosine_gemm_only_ms'], 'norms', d['row_norms_ms'], 'ref', d['reference_recipe_cosine_ms'])"
