#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_oneshot_gpu.py tests/test_ddp.py tests/test_engine_gpu.py tests/test_graphed_compute_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_s40_tests.log 2>&1 || { tail -30 gpurun_out/r3_s40_tests.log; exit 1; }
tail -1 gpurun_out/r3_s40_tests.log
