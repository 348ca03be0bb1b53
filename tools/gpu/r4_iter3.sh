#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 120 python benchmarks/bench_atomics.py > gpurun_out/r4i3_atomics.jsonl 2>gpurun_out/r4i3_atomics.err || { tail -20 gpurun_out/r4i3_atomics.err; exit 1; }
cat gpurun_out/r4i3_atomics.jsonl | tr -d '{}"' | paste -sd' ' | fold -w 3000
T="tests/test_fused_compute_gpu.py tests/test_macro_curves.py tests/test_native_forward_gpu.py tests/test_gemm_big_gpu.py tests/test_torchscript.py tests/test_regression.py tests/test_native_update.py tests/test_state_arena.py tests/test_forward_aliasing.py"
timeout -k 10 400 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i3_pytest.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4i3_pytest.log | head -30
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 300 python benchmarks/bench_forward.py 2>gpurun_out/r4i3_forward.err > gpurun_out/r4i3_bench_forward.jsonl || { tail -20 gpurun_out/r4i3_forward.err; exit 1; }
cut -c1-330 gpurun_out/r4i3_bench_forward.jsonl
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step 2>gpurun_out/r4i3_collection.err > gpurun_out/r4i3_collection.json || { tail -20 gpurun_out/r4i3_collection.err; exit 1; }
cut -c1-500 gpurun_out/r4i3_collection.json
