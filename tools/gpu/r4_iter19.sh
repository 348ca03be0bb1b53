#!/bin/bash
# few-class tile kernel: kernel time with the flush / the row work switched off (TM_AMD_FEWBINS_DEBUG)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp
for kind in confmat acc; do
  for dbg in 0 1 2 3; do
    for tile in 2 4; do
      d=$R/gpurun_out/fb_${kind}_${dbg}_${tile}
      FEWBINS_KIND=$kind TM_AMD_FEWBINS_DEBUG=$dbg TM_AMD_FEWBINS_TILE=$tile timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o p -- python3 $R/benchmarks/fewbins_one.py > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
      echo "$kind dbg=$dbg tile=$tile $(python3 $R/tools/gpu/trace_summary.py $d --match fewbins | cut -c1-160 | tail -2 | tr '\n' ' ')"
      rm -rf $d
    done
  done
done
