#!/bin/bash
# Round 5: the driver's exact headline command, 5 fresh processes, then a per-dispatch timeline
# (kernel trace + HIP runtime trace) of the same command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
for i in 1 2 3 4 5; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_b20_$i.log 2>&1 || { tail -20 gpurun_out/r5_b20_$i.log; exit 1; }
  grep '^{' gpurun_out/r5_b20_$i.log | cut -c1-200
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/r5tl -o tl -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-baseline > $R/gpurun_out/r5tl.log 2>&1 || { tail -20 $R/gpurun_out/r5tl.log; exit 1; }
cd $R && grep '^{' gpurun_out/r5tl.log | cut -c1-200
find gpurun_out/r5tl -name "*.csv" | xargs ls -la
