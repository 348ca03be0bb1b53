#!/bin/bash
# Round 5: compute()'s validation read through mapped memory + stream sync; headline x7; GPU tests touching it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_native_update.py tests/test_native_forward_gpu.py tests/test_fused_compute_gpu.py tests/test_stream_kernels_gpu.py tests/test_determinism_gpu.py tests/test_engine_gpu.py -m gpu > gpurun_out/r5rw_tests.log 2>&1 || { tail -30 gpurun_out/r5rw_tests.log; exit 1; }
tail -2 gpurun_out/r5rw_tests.log
for i in 1 2 3 4 5 6 7; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5rw_b20_$i.log 2>&1 || { tail -20 gpurun_out/r5rw_b20_$i.log; exit 1; }
  grep '^{' gpurun_out/r5rw_b20_$i.log >> gpurun_out/r5rw_bench20.jsonl
  grep -o '"value": [0-9.]*' gpurun_out/r5rw_b20_$i.log | head -1
done
timeout -k 10 120 python3 benchmarks/first_region_probe.py onering > gpurun_out/r5rw_probe.jsonl 2>&1 || exit 1
cut -c1-300 gpurun_out/r5rw_probe.jsonl
