#!/bin/bash
# Refresh the committed evidence under profiles/: headline bench + rocprof kernel stats, config #3/#4/#5 benches.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/p
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 500 --warmup 50 > gpurun_out/p/bench.json 2> gpurun_out/p/bench.err || exit 1
tail -1 gpurun_out/p/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p/bprof -o b --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-baseline > $R/gpurun_out/p/bprof.log 2>&1 || exit 1
cd $R
timeout -k 10 300 python benchmarks/bench_collection.py --steps 300 --warmup 30 > gpurun_out/p/coll.jsonl 2>&1 || exit 1
timeout -k 10 300 python benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step >> gpurun_out/p/coll.jsonl 2>&1 || exit 1
timeout -k 10 300 python benchmarks/bench_collection.py --steps 300 --warmup 30 --graph >> gpurun_out/p/coll.jsonl 2>&1 || exit 1
grep -v amdgpu gpurun_out/p/coll.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p/cprof -o c --output-format csv -- python3 $R/benchmarks/bench_collection.py --steps 100 --warmup 10 > $R/gpurun_out/p/cprof.log 2>&1 || exit 1
cd $R
timeout -k 10 600 python benchmarks/bench_fid.py > gpurun_out/p/fid.log 2>&1 || exit 1
tail -1 gpurun_out/p/fid.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p/fprof -o f --output-format csv -- python3 $R/benchmarks/bench_fid.py > $R/gpurun_out/p/fprof.log 2>&1 || exit 1
cd $R
timeout -k 10 600 python benchmarks/bench_map.py > gpurun_out/p/map.log 2>&1 || exit 1
tail -2 gpurun_out/p/map.log
