#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step > gpurun_out/r3_s21_coll_sync.json 2>&1 || { tail -30 gpurun_out/r3_s21_coll_sync.json; exit 1; }
tail -1 gpurun_out/r3_s21_coll_sync.json
timeout -k 10 300 python -u benchmarks/bench_collection.py --steps 300 --warmup 30 > gpurun_out/r3_s21_coll.json 2>&1 || { tail -30 gpurun_out/r3_s21_coll.json; exit 1; }
tail -1 gpurun_out/r3_s21_coll.json
timeout -k 10 300 python -u benchmarks/collection_compute_eager.py > gpurun_out/r3_s21_coll_eager.json 2>&1 || { tail -30 gpurun_out/r3_s21_coll_eager.json; exit 1; }
cat gpurun_out/r3_s21_coll_eager.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_s21_prof -o coll -- python3 $GRAFT_REPO_ROOT/benchmarks/collection_compute_eager.py --loop 100 > $GRAFT_REPO_ROOT/gpurun_out/r3_s21_prof.txt 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/r3_s21_prof.txt; exit 1; }
