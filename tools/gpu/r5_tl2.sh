#!/bin/bash
# Round 5: where the first timed region goes.  (1) kernel trace only (light) of the exact driver command;
# (2) host-phase probe in fresh processes: bench's ring, then the same with the region reading only the 5 warm slots.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5kt -o kt -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-baseline > $R/gpurun_out/r5kt.log 2>&1 || { tail -20 $R/gpurun_out/r5kt.log; exit 1; }
cd $R && grep '^{' gpurun_out/r5kt.log | cut -c1-200
for c in onering onering_same5 onering onering_same5 warm50; do
  timeout -k 10 120 python3 benchmarks/first_region_probe.py $c >> gpurun_out/r5_first_region.jsonl 2>gpurun_out/r5_fr.err || { tail -5 gpurun_out/r5_fr.err; exit 1; }
done
cut -c1-160 gpurun_out/r5_first_region.jsonl
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --ring-mb 64 --no-baseline > gpurun_out/r5_b20_ring64_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/r5_b20_ring64_$i.log | cut -c1-160
done
