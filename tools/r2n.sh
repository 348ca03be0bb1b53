#!/bin/bash
# GPU step: calibration cache tests + config #5 bench with per-step compute
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH="$R"

timeout -k 10 300 python -u benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step --graph > gpurun_out/r2n_coll.json 2>&1 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2n_prof -o p --output-format csv -- python3 $R/benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step --graph > $R/gpurun_out/r2n_prof.log 2>&1) &&
timeout -k 10 300 python -u benchmarks/bench_map.py > gpurun_out/r2n_map.json 2>&1
