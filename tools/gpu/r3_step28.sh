#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_sklearn_pinned_gpu.py > gpurun_out/r3_s28_tests.log 2>&1 || { tail -40 gpurun_out/r3_s28_tests.log; exit 1; }
tail -3 gpurun_out/r3_s28_tests.log
