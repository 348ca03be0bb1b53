#!/bin/bash
# GPU step: ranking kernel tests + config #5 re-measure + mAP bench
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH="$R"
timeout -k 10 300 python -u -m pytest tests/test_ranking_gpu.py tests/test_calibration_cache_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2o_tests.log 2>&1 &&
bash tools/r2n.sh
