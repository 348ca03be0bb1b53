#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
for case in plain sched_spin sched_yield sched_blocking plain sched_spin sched_yield sched_blocking; do
  timeout -k 10 120 python -u benchmarks/first_region_probe.py $case 2>/dev/null | tee -a gpurun_out/r3_first_region2.jsonl || exit 1
done
