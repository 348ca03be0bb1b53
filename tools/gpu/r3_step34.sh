#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dgemm_gpu.py tests/test_image_generative.py -m gpu > gpurun_out/r3_s34_tests.log 2>&1 || { tail -40 gpurun_out/r3_s34_tests.log; exit 1; }
tail -2 gpurun_out/r3_s34_tests.log
timeout -k 10 300 python -u benchmarks/bench_fid.py > gpurun_out/r3_s34_fid.json 2>&1 || { tail -30 gpurun_out/r3_s34_fid.json; exit 1; }
tail -1 gpurun_out/r3_s34_fid.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_s34_prof -o fid -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_fid.py --no-baseline > $GRAFT_REPO_ROOT/gpurun_out/r3_s34_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_s34_prof.log; exit 1; }
