#!/bin/bash
# launch-path warm-up probe: fresh process per run, prelaunch 0 / 64 / 512 / 4096 tiny kernels, 3 runs each
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
: > gpurun_out/r3_launch_warm_probe.jsonl
for rep in 1 2 3; do
  for n in 0 64 512 4096; do
    timeout -k 10 120 python benchmarks/launch_warm_probe.py --prelaunch $n 2>/dev/null >> gpurun_out/r3_launch_warm_probe.jsonl || exit 1
  done
done
cut -c1-200 gpurun_out/r3_launch_warm_probe.jsonl
