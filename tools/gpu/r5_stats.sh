#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
for m in 1 2 4; do
  TM_AMD_BIN_VEC_BLOCKS_PER_CU=$m timeout -k 10 200 python3 benchmarks/bench_binary_stats.py > gpurun_out/r5s_stats_$m.jsonl 2>&1 || { tail -5 gpurun_out/r5s_stats_$m.jsonl; exit 1; }
  echo "blocks/CU=$m"; grep -h "Multilabel" gpurun_out/r5s_stats_$m.jsonl
done
