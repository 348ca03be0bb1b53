#!/bin/bash
# dgemm wave-count sweep + short-region breakdown of the headline with the native update.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
bash tools/gpu/tests.sh dgemm_tests tests/test_dgemm_gpu.py || exit 1
for w in 4 8; do
  TM_AMD_DGEMM_WAVES=$w timeout -k 10 300 python -u benchmarks/bench_dgemm.py >> gpurun_out/r3_bench_dgemm_sweep.jsonl 2> gpurun_out/r3_bench_dgemm.err || { tail -20 gpurun_out/r3_bench_dgemm.err; exit 1; }
done
cat gpurun_out/r3_bench_dgemm_sweep.jsonl
timeout -k 10 300 python -u benchmarks/short_region_probe.py > gpurun_out/r3_short_region.json 2>&1 || { tail -20 gpurun_out/r3_short_region.json; exit 1; }
cat gpurun_out/r3_short_region.json
bash tools/gpu/tests.sh fid_tests tests/test_image_generative.py || exit 1
timeout -k 10 600 python -u benchmarks/bench_fid.py > gpurun_out/r3_bench_fid.jsonl 2> gpurun_out/r3_bench_fid.err || { tail -20 gpurun_out/r3_bench_fid.err; exit 1; }
cat gpurun_out/r3_bench_fid.jsonl
timeout -k 10 300 python -u benchmarks/fid_ns_breakdown.py > gpurun_out/r3_fid_ns_breakdown.json 2>&1 || { tail -20 gpurun_out/r3_fid_ns_breakdown.json; exit 1; }
grep -v amdgpu gpurun_out/r3_fid_ns_breakdown.json
