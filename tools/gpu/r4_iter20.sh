#!/bin/bash
# few-class tile kernel with per-block partials + fold: correctness, then kernel time per blocks-per-CU
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stream_kernels_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/r4i20_tests.log 2>&1 || { tail -30 gpurun_out/r4i20_tests.log; exit 1; }
tail -2 gpurun_out/r4i20_tests.log
cd /tmp
for kind in confmat acc; do
  for cfg in "2 0" "2 1" "3 1" "4 1" "8 1"; do
    set -- $cfg
    d=$R/gpurun_out/fb_${kind}_$1_$2
    FEWBINS_KIND=$kind TM_AMD_FEWBINS_TILE=$1 TM_AMD_FEWBINS_FOLD=$2 timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o p -- python3 $R/benchmarks/fewbins_one.py > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    echo "$kind tile=$1 fold=$2"; python3 $R/tools/gpu/trace_summary.py $d --match _kernel | cut -c1-150 | grep -v "^$" | head -6
    rm -rf $d
  done
done
