#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5fs_smoke.log 2>&1 || { tail -30 gpurun_out/r5fs_smoke.log; exit 1; }
tail -1 gpurun_out/r5fs_smoke.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_regression.py tests/test_fused_compute_gpu.py -m gpu > gpurun_out/r5fs_tests.log 2>&1 || { tail -30 gpurun_out/r5fs_tests.log; exit 1; }
tail -1 gpurun_out/r5fs_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5fs_bench.log 2>&1 || { tail -30 gpurun_out/r5fs_bench.log; exit 1; }
grep '^{' gpurun_out/r5fs_bench.log | cut -c1-160
