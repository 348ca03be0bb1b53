#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
TM_AMD_GEMM16_PERSIST=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_h16_gpu.py tests/test_pairwise.py -m gpu > gpurun_out/r5g7_tests.log 2>&1 || { tail -30 gpurun_out/r5g7_tests.log; exit 1; }
tail -1 gpurun_out/r5g7_tests.log
for p in 0 1 2; do
  TM_AMD_GEMM16_PERSIST=$p timeout -k 10 200 python3 benchmarks/bench_gemm16.py > gpurun_out/r5g7_bench_$p.jsonl 2>&1 || { tail -5 gpurun_out/r5g7_bench_$p.jsonl; exit 1; }
  echo "persist=$p"
  grep -h shape gpurun_out/r5g7_bench_$p.jsonl | grep bfloat16 | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(' ', d['shape'], 'store', d['store_ms'], 'blt', d['hipblaslt_ms'], 'cos', d['pairwise_cosine_ms'], 'ref', d['reference_recipe_cosine_ms'])"
done
