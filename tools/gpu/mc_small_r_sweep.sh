#!/bin/bash
# Rows-per-thread (tile size) x blocks-per-CU sweep of the few-class tile kernel with the group hand-off:
# bench_mc_small.py wall clock per variant, then kernel statistics of each variant.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=("TM_AMD_FEWBINS_R=6" "TM_AMD_FEWBINS_R=4" "TM_AMD_FEWBINS_R=3" "TM_AMD_FEWBINS_R=2" "TM_AMD_FEWBINS_R=3 TM_AMD_FEWBINS_TILE=2" "TM_AMD_FEWBINS_R=2 TM_AMD_FEWBINS_TILE=2" "TM_AMD_FEWBINS_R=6 TM_AMD_FEWBINS_TILE=4")
for v in "${V[@]}"; do
  ( export $v CLASSES=4,10 && timeout -k 10 120 python3 -u benchmarks/bench_mc_small.py >> gpurun_out/mcr_bench.jsonl 2>> gpurun_out/mcr_bench.err ) || { echo "variant $v failed"; tail -20 gpurun_out/mcr_bench.err; exit 1; }
done
cat gpurun_out/mcr_bench.jsonl
bash tools/gpu/kstat_sweep.sh mcr benchmarks/bench_mc_small.py fewbins "${V[@]}"
