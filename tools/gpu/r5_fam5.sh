#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider "tests/test_fused_update_gpu.py::test_fused_update_group_widths" -m gpu > gpurun_out/r5f5_tests.log 2>&1; rc=$?
grep -E "^FAILED|passed|failed|Mismatch|Greatest" gpurun_out/r5f5_tests.log | head -40
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
