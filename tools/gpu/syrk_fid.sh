#!/bin/bash
# SYRK sweep (feature statistics) + fp64 GEMM bench + FID bench line + ours-only FID kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
N=${1:-sf}
timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_dgemm_gpu.py tests/test_image_generative.py -m gpu > gpurun_out/${N}_tests.log 2>&1 || { tail -30 gpurun_out/${N}_tests.log; exit 1; }
tail -1 gpurun_out/${N}_tests.log
timeout -k 10 300 python benchmarks/syrk_sweep.py > gpurun_out/${N}_syrk.jsonl 2>&1 || { tail -20 gpurun_out/${N}_syrk.jsonl; exit 1; }
grep '"auto"\|reference' gpurun_out/${N}_syrk.jsonl
bash tools/gpu/fid_prof.sh ${N}
