#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
for bk in 32 64; do for st in 1 2; do
  TM_AMD_GEMM_BK=$bk TM_AMD_GEMM_STAGES=$st timeout -k 10 200 python -u benchmarks/gemm_sweep.py >> gpurun_out/r3_s32_sweep.jsonl 2>&1 || { tail -20 gpurun_out/r3_s32_sweep.jsonl; exit 1; }
done; done
grep shape gpurun_out/r3_s32_sweep.jsonl
