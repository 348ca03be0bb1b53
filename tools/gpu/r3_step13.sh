#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
for i in 1 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_s13_bench20_$i.log 2>&1 || { tail -30 gpurun_out/r3_s13_bench20_$i.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/r3_s13_bench20_$i.log | tr '\n' ' '; echo
done
timeout -k 10 300 python -u bench.py > gpurun_out/r3_s13_bench200.log 2>&1 || { tail -30 gpurun_out/r3_s13_bench200.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3_s13_bench200.log | tr '\n' ' '; echo
