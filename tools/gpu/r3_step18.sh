#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_collection_checks_gpu.py tests/test_kernels_gpu.py tests/test_graphed_compute_gpu.py tests/test_engine_gpu.py tests/test_oneshot_gpu.py -m gpu > gpurun_out/r3_s18_tests.log 2>&1 || { tail -40 gpurun_out/r3_s18_tests.log; exit 1; }
tail -3 gpurun_out/r3_s18_tests.log
timeout -k 10 300 python -u benchmarks/collection_compute_eager.py > gpurun_out/r3_s18_coll_eager.json 2>&1 || { tail -30 gpurun_out/r3_s18_coll_eager.json; exit 1; }
cat gpurun_out/r3_s18_coll_eager.json
