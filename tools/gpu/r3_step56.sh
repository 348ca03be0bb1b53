#!/bin/bash
# final-build 1-GPU runs of BASELINE configs #3 (mAP) and #4 (FID)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 400 python benchmarks/bench_map.py 2>/dev/null > gpurun_out/r3_bench_map_final.json || exit 1
tail -1 gpurun_out/r3_bench_map_final.json | cut -c1-300
timeout -k 10 600 python benchmarks/bench_fid.py 2>/dev/null > gpurun_out/r3_bench_fid_final.json || exit 1
tail -1 gpurun_out/r3_bench_fid_final.json | cut -c1-400
