#!/bin/bash
# Round-3 starting point: three short headline runs and the host-side update profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench20_$i.log 2>&1 || { tail -30 gpurun_out/r3_bench20_$i.log; exit 1; }
  grep metric gpurun_out/r3_bench20_$i.log
done
timeout -k 10 300 python -u benchmarks/host_update_profile.py > gpurun_out/r3_host_profile.log 2>&1 || { tail -30 gpurun_out/r3_host_profile.log; exit 1; }
head -40 gpurun_out/r3_host_profile.log
