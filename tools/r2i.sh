#!/bin/bash
# GPU step: reduced-precision tests through the HIP kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_precision_grad.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2i_precision.log 2>&1
