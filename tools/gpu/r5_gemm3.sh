#!/bin/bash
# 16-bit GEMM: 4-wave 128x128-per-wave kernel (TM_AMD_GEMM16_W4=1) vs the 8-wave kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
TM_AMD_GEMM16_W4=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_h16_gpu.py -m gpu > gpurun_out/r5g3_tests.log 2>&1 || { tail -30 gpurun_out/r5g3_tests.log; exit 1; }
tail -1 gpurun_out/r5g3_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_h16_gpu.py tests/test_pairwise.py -m gpu > gpurun_out/r5g3_tests0.log 2>&1 || { tail -30 gpurun_out/r5g3_tests0.log; exit 1; }
tail -1 gpurun_out/r5g3_tests0.log
for w in 0 1; do
  TM_AMD_GEMM16_W4=$w timeout -k 10 200 python3 benchmarks/bench_gemm16.py > gpurun_out/r5g3_bench_w$w.jsonl 2>&1 || { tail -5 gpurun_out/r5g3_bench_w$w.jsonl; exit 1; }
  echo "W4=$w"; grep shape gpurun_out/r5g3_bench_w$w.jsonl | grep bfloat16 | cut -c1-200
done
grep -h shape gpurun_out/r5g3_bench_w0.jsonl | grep bfloat16 | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], 'cos', d['pairwise_cosine_ms'], 'ref', d['reference_recipe_cosine_ms'])"
