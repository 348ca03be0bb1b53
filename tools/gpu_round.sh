#!/bin/bash
# One gpurun session: GPU tests, smoke, bench, rocprof kernel stats. Each GPU step has its own time limit and the
# chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
if [[ $STEP == all || $STEP == test || $STEP == quick ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STEP == all || $STEP == smoke ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -40 gpurun_out/smoke.log; exit 1; }
  tail -2 gpurun_out/smoke.log
fi
if [[ $STEP == all || $STEP == bench || $STEP == quick ]]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -40 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log
fi
if [[ $STEP == all || $STEP == prof ]]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { tail -40 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  find gpurun_out/prof -name "*kernel_stats*" | head -3
fi
if [[ $STEP == all || $STEP == kbench || $STEP == quick ]]; then
  timeout -k 10 300 python benchmarks/kbench.py > gpurun_out/kbench.log 2>&1 || { tail -40 gpurun_out/kbench.log; exit 1; }
  cat gpurun_out/kbench.log
fi
if [[ $STEP == kprof ]]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/kprof -o kb --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/kbench.py > $GRAFT_REPO_ROOT/gpurun_out/kprof.log 2>&1 || { tail -40 $GRAFT_REPO_ROOT/gpurun_out/kprof.log; exit 1; }
  cd $GRAFT_REPO_ROOT && cut -c1-200 gpurun_out/kprof/kb_kernel_stats.csv | head -30
fi
if [[ $STEP == tune ]]; then
  timeout -k 10 120 python benchmarks/host_overhead.py 2>&1 | grep -v amdgpu.ids
  for L in 8 16 32 64; do
    cd /tmp && TM_AMD_MC_LPR=$L timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/tune$L -o t --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/kbench.py --N 8192 --C 1000 > /dev/null 2>&1 || exit 1
    cd $GRAFT_REPO_ROOT
  done
fi
if [[ $STEP == fid ]]; then
  timeout -k 10 900 python -m pytest tests/test_image_generative.py -m gpu -x -q > gpurun_out/pytest_fid.log 2>&1 || { tail -40 gpurun_out/pytest_fid.log; exit 1; }
  tail -2 gpurun_out/pytest_fid.log
  timeout -k 10 900 python benchmarks/bench_fid.py > gpurun_out/bench_fid.log 2>&1 || { tail -40 gpurun_out/bench_fid.log; exit 1; }
  tail -1 gpurun_out/bench_fid.log
fi
if [[ $STEP == fidprof ]]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fidprof -o f --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_fid.py > $GRAFT_REPO_ROOT/gpurun_out/fidprof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/fidprof.log; exit 1; }
fi
