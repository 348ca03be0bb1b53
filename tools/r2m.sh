#!/bin/bash
# GPU step: boundary tests + regression kernels
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH="$R"
timeout -k 10 500 python -u -m pytest tests/test_kernel_boundaries_gpu.py tests/test_regression.py tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2m_tests.log 2>&1
