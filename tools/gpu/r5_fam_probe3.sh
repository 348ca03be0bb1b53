#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp
for ab in 0 32 1 2 4 8 16 22; do
  TM_AMD_FAMILY_ABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fp3 -o p -- python3 $R/benchmarks/family_probe.py > $R/gpurun_out/fp3.log 2>&1 || { tail -5 $R/gpurun_out/fp3.log; exit 1; }
  echo "ablate=$ab $(grep step_us $R/gpurun_out/fp3.log | cut -c1-60) $(python3 $R/tools/gpu/kstats.py $R/gpurun_out/fp3 family_rows | cut -c73-)"
  rm -rf $R/gpurun_out/fp3
done
