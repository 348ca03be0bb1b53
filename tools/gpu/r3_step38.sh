#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_oneshot_gpu.py tests/test_ddp.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_s38_tests.log 2>&1 || { tail -30 gpurun_out/r3_s38_tests.log; exit 1; }
tail -1 gpurun_out/r3_s38_tests.log
