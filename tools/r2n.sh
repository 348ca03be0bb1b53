#!/bin/bash
# GPU step: calibration cache tests + config #5 bench with per-step compute
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH="$R"
timeout -k 10 300 python -u -m pytest tests/test_calibration_cache_gpu.py tests/test_graphed_compute_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2n_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step --graph > gpurun_out/r2n_coll.json 2>&1
