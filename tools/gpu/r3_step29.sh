#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u benchmarks/bench_gemm.py > gpurun_out/r3_s29_gemm.jsonl 2>&1 || { tail -30 gpurun_out/r3_s29_gemm.jsonl; exit 1; }
cat gpurun_out/r3_s29_gemm.jsonl
timeout -k 10 300 python -u benchmarks/bench_pairwise.py > gpurun_out/r3_s29_pairwise.jsonl 2>&1 || { tail -30 gpurun_out/r3_s29_pairwise.jsonl; exit 1; }
grep -E "linear|cosine" gpurun_out/r3_s29_pairwise.jsonl
