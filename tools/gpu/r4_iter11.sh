#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_clustering_gpu.py tests/test_clustering.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i11_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed|^E  " gpurun_out/r4i11_pytest.log | head -20
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 300 python benchmarks/bench_clustering.py --ours-only > gpurun_out/r4i11_clustering.jsonl 2>gpurun_out/r4i11_clu.err || { tail -20 gpurun_out/r4i11_clu.err; exit 1; }
cat gpurun_out/r4i11_clustering.jsonl
timeout -k 10 300 python benchmarks/bench_clustering.py > gpurun_out/r4i11_clustering_vs_ref.jsonl 2>gpurun_out/r4i11_clu2.err || { tail -20 gpurun_out/r4i11_clu2.err; exit 1; }
cat gpurun_out/r4i11_clustering_vs_ref.jsonl
