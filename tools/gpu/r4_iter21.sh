#!/bin/bash
# few-class tile kernel + split fold: correctness, kernel times, stats-update bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stream_kernels_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/r4i21_tests.log 2>&1 || { tail -30 gpurun_out/r4i21_tests.log; exit 1; }
tail -1 gpurun_out/r4i21_tests.log
cd /tmp
for cfg in "acc 3 10" "confmat 3 10" "acc 3 4" "acc 3 8" "acc 3 16" "acc 3 32" "confmat 3 32" "acc 3 64"; do
  set -- $cfg
  d=$R/gpurun_out/fb_$1_$2_$3
  FEWBINS_KIND=$1 TM_AMD_FEWBINS_TILE=$2 FEWBINS_C=$3 timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o p -- python3 $R/benchmarks/fewbins_one.py > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "$1 tile=$2 C=$3"; python3 $R/tools/gpu/trace_summary.py $d --match _kernel | cut -c1-150 | grep -v "^$" | grep "fewbins\|finalize\|mc_"
  rm -rf $d
done
cd $R
for t in 3; do TM_AMD_FEWBINS_TILE=$t timeout -k 10 200 python benchmarks/bench_binary_stats.py > gpurun_out/r4i21_stats_$t.jsonl 2>&1 || { tail -5 gpurun_out/r4i21_stats_$t.jsonl; exit 1; }; echo "tile $t"; cat gpurun_out/r4i21_stats_$t.jsonl; done
