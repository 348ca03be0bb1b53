#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
TM_AMD_GEMM16_RING=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_h16_gpu.py -m gpu > gpurun_out/r5g5_tests.log 2>&1 || { tail -30 gpurun_out/r5g5_tests.log; exit 1; }
tail -1 gpurun_out/r5g5_tests.log
for cfg in "0 -1" "2 -1" "1 -1" "0 0"; do
  set -- $cfg
  if [ "$2" = "-1" ]; then unset TM_AMD_GEMM16_BIG; else export TM_AMD_GEMM16_BIG=$2; fi
  TM_AMD_GEMM16_RING=$1 timeout -k 10 200 python3 benchmarks/bench_gemm16.py > gpurun_out/r5g5_bench.jsonl 2>&1 || { tail -5 gpurun_out/r5g5_bench.jsonl; exit 1; }
  echo "ring=$1 big=$2"
  grep -h shape gpurun_out/r5g5_bench.jsonl | grep bfloat16 | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(' ', d['shape'], 'store', d['store_ms'], 'blt', d['hipblaslt_ms'], 'cos', d['pairwise_cosine_ms'], 'ref', d['reference_recipe_cosine_ms'])"
done
