#!/bin/bash
# Round-2 GPU steps: targeted tests, a benchmark and its rocprofv3 kernel stats.  Each GPU step has its own time
# limit; the chain stops at the first failure.
#   bash tools/gpu_step.sh "<pytest files or -k expr>" <bench script or ''> [prof]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TESTS=$1
BENCH=$2
PROF=$3
if [[ -n "$TESTS" ]]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_step.log 2>&1 || { tail -60 gpurun_out/pytest_step.log; exit 1; }
  tail -3 gpurun_out/pytest_step.log
fi
if [[ -n "$BENCH" ]]; then
  timeout -k 10 600 python $BENCH > gpurun_out/bench_step.log 2>&1 || { tail -40 gpurun_out/bench_step.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/bench_step.log
  if [[ -n "$PROF" ]]; then
    cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_step -o p --output-format csv -- python3 $R/$BENCH > $R/gpurun_out/prof_step.log 2>&1 || { tail -30 $R/gpurun_out/prof_step.log; exit 1; }
    cd $R && cp gpurun_out/prof_step/*/p_kernel_stats.csv gpurun_out/prof_step_kernel_stats.csv 2>/dev/null || cp $(find gpurun_out/prof_step -name "*kernel_stats.csv" | head -1) gpurun_out/prof_step_kernel_stats.csv
    rm -rf gpurun_out/prof_step
    cut -d, -f1-4 gpurun_out/prof_step_kernel_stats.csv | head -25
  fi
fi
