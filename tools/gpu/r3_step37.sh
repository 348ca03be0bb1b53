#!/bin/bash
# Narrow-wire sync with CUDA tensors (2 processes, one device), tiled CLIP-IQA kernel, retrieval / CLIP bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_ddp.py tests/test_multimodal.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_s37_tests.log 2>&1 || { tail -30 gpurun_out/r3_s37_tests.log; exit 1; }
tail -1 gpurun_out/r3_s37_tests.log
timeout -k 10 300 python benchmarks/bench_retrieval_clip.py > gpurun_out/r3_bench_retrieval_clip.jsonl 2>&1 || { tail -20 gpurun_out/r3_bench_retrieval_clip.jsonl; exit 1; }
grep -v amdgpu.ids gpurun_out/r3_bench_retrieval_clip.jsonl
