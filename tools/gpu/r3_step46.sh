#!/bin/bash
# config #5 collection after the setattr / reset changes: eager compute every step, update only, HIP-graph compute
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step 2>/dev/null > gpurun_out/r3_collection_sync_every_step.json || exit 1
cut -c1-260 gpurun_out/r3_collection_sync_every_step.json
timeout -k 10 300 python benchmarks/bench_collection.py --steps 300 --warmup 30 2>/dev/null > gpurun_out/r3_collection_bench.json || exit 1
cut -c1-260 gpurun_out/r3_collection_bench.json
timeout -k 10 300 python benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step --graph --no-baseline 2>/dev/null > gpurun_out/r3_collection_graphed.json || exit 1
cut -c1-260 gpurun_out/r3_collection_graphed.json
