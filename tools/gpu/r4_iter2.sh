#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/gpu/diag_forward.py > gpurun_out/r4i2_diag_forward.log 2>&1 || { tail -30 gpurun_out/r4i2_diag_forward.log; exit 1; }
grep "after call" gpurun_out/r4i2_diag_forward.log
timeout -k 10 60 python tools/gpu/diag_interp.py > gpurun_out/r4i2_diag_interp.log 2>&1 || { tail -30 gpurun_out/r4i2_diag_interp.log; exit 1; }
head -3 gpurun_out/r4i2_diag_interp.log
T="tests/test_fused_compute_gpu.py tests/test_macro_curves.py tests/test_native_forward_gpu.py tests/test_gemm_big_gpu.py tests/test_torchscript.py tests/test_regression.py"
timeout -k 10 400 python -u -m pytest $T -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i2_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed|^E  " gpurun_out/r4i2_pytest.log | head -30
exit $rc
