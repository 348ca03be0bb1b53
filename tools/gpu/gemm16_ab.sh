#!/bin/bash
# 16-bit GEMM: GPU tests, then bench_gemm16.py with the ping-pong main loop on / off (TM_AMD_GEMM16_PP).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
N=${1:-g16}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_h16_gpu.py tests/test_bert_match_gpu.py > gpurun_out/${N}_tests.log 2>&1 || { tail -30 gpurun_out/${N}_tests.log; exit 1; }
tail -1 gpurun_out/${N}_tests.log
for pp in ${PPS:-1 0}; do
  TM_AMD_GEMM16_PP=$pp timeout -k 10 300 python benchmarks/bench_gemm16.py > gpurun_out/${N}_bench_pp$pp.jsonl 2>&1 || { tail -20 gpurun_out/${N}_bench_pp$pp.jsonl; exit 1; }
  echo "pp=$pp"; grep '^{' gpurun_out/${N}_bench_pp$pp.jsonl | cut -c1-170
done
