#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_coll -o p -- python3 $R/benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step --no-baseline > $R/gpurun_out/r4i7_coll.log 2>&1 || { tail -20 $R/gpurun_out/r4i7_coll.log; exit 1; }
cd $R && python3 tools/gpu/trace_summary.py gpurun_out/prof_coll --calls 111 > gpurun_out/r4i7_coll_trace.txt && head -30 gpurun_out/r4i7_coll_trace.txt | cut -c1-140 && rm -rf gpurun_out/prof_coll
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_fb -o p -- python3 $R/benchmarks/bench_fewbins.py > $R/gpurun_out/r4i7_fb.log 2>&1 || { tail -20 $R/gpurun_out/r4i7_fb.log; exit 1; }
cd $R && python3 tools/gpu/trace_summary.py gpurun_out/prof_fb --match tm_amd | cut -c1-140 && rm -rf gpurun_out/prof_fb
