#!/bin/bash
# confmat ring microbenchmark + 1-GPU runs of the config #3/#4/#5 benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 120 ./tools/mb/confmat_ring_mb > gpurun_out/r3_confmat_ring_mb.jsonl 2>&1 || { tail -20 gpurun_out/r3_confmat_ring_mb.jsonl; exit 1; }
cat gpurun_out/r3_confmat_ring_mb.jsonl
timeout -k 10 300 python -u benchmarks/bench_fid.py > gpurun_out/r3_bench_fid1.json 2> gpurun_out/r3_bench_fid1.err || { tail -20 gpurun_out/r3_bench_fid1.err; exit 1; }
cat gpurun_out/r3_bench_fid1.json
timeout -k 10 300 python -u benchmarks/bench_map.py > gpurun_out/r3_bench_map1.json 2> gpurun_out/r3_bench_map1.err || { tail -20 gpurun_out/r3_bench_map1.err; exit 1; }
cat gpurun_out/r3_bench_map1.json
timeout -k 10 300 python -u benchmarks/bench_collection.py --sync-every-step > gpurun_out/r3_bench_coll1.json 2> gpurun_out/r3_bench_coll1.err || { tail -20 gpurun_out/r3_bench_coll1.err; exit 1; }
cat gpurun_out/r3_bench_coll1.json
