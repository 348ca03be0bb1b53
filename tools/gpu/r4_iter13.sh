#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gemm_big_gpu.py tests/test_gemm_kernels.py tests/test_gemm_rowcolmax_gpu.py tests/test_pairwise.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i13_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i13_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
for pipe in 1 0; do
  TM_AMD_GEMM_PIPE=$pipe timeout -k 10 300 python benchmarks/bench_gemm.py > gpurun_out/r4i13_gemm_pipe$pipe.jsonl 2>gpurun_out/r4i13_gemm.err || { tail -20 gpurun_out/r4i13_gemm.err; exit 1; }
  echo "== pipe $pipe"; python3 -c "
import json
for l in open('gpurun_out/r4i13_gemm_pipe$pipe.jsonl'):
    d=json.loads(l); print(d['shape'], 'store', d['store_ms'], d['store_tflops'], 'hipblaslt', d['hipblaslt_mm_ms'], d['hipblaslt_tflops'], 'rowmin', d['fused_rowmin_ms'], 'polysum', d['fused_polysum_ms'])
"
done
