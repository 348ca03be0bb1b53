#!/bin/bash
# headline kernel grid: blocks per CU (1 row per wave at 4; 2 / 4 rows per wave at 2 / 1, double-buffered)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
for m in 4 2 1 3; do
  for i in 1 2; do
    TM_AMD_ORD16_BLOCKS_PER_CU=$m timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5o_$m_$i.log 2>&1 || { tail -5 gpurun_out/r5o_$m_$i.log; exit 1; }
    echo "per_cu=$m $(grep '^{' gpurun_out/r5o_$m_$i.log | cut -c1-110)"
  done
  cd /tmp && TM_AMD_ORD16_BLOCKS_PER_CU=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/o -o p -- python3 $R/bench.py --steps 200 --warmup 20 --no-baseline > $R/gpurun_out/o.log 2>&1 || { tail -5 $R/gpurun_out/o.log; exit 1; }
  cd $R && echo "per_cu=$m $(python3 tools/gpu/kstats.py gpurun_out/o ord16 | cut -c60-)"; rm -rf gpurun_out/o
done
