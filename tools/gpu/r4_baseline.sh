#!/bin/bash
# Round-4 GPU call: this round's new GPU tests first, then the full GPU suite, smoke, two fresh 20-step headline runs
# and the benches of this round's work.  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
NEW="tests/test_native_forward_gpu.py tests/test_native_update.py tests/test_stream_kernels_gpu.py tests/test_macro_curves.py tests/test_iou_module.py tests/test_fused_compute_gpu.py tests/test_functional_kernels_gpu.py tests/test_torchscript.py tests/test_audio.py tests/test_gemm_big_gpu.py"
timeout -k 10 400 python -u -m pytest $NEW -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pytest_new.log 2>&1; rc=$?
tail -30 gpurun_out/r4_pytest_new.log | grep -E "FAILED|ERROR|passed|failed|error" | head -40
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc   # 1 = test failures: keep going to collect the rest; anything else stops
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider --deselect tests/test_gemm_big_gpu.py > gpurun_out/r4_pytest_gpu.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r4_pytest_gpu.log | tail -30
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -30 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench20_$i.log 2>&1 || { tail -30 gpurun_out/r4_bench20_$i.log; exit 1; }
  grep '^{' gpurun_out/r4_bench20_$i.log | cut -c1-220
done
timeout -k 10 300 python benchmarks/bench_forward.py 2>/dev/null > gpurun_out/r4_bench_forward.jsonl || exit 1
cat gpurun_out/r4_bench_forward.jsonl
timeout -k 10 300 python benchmarks/bench_binary_stats.py 2>/dev/null > gpurun_out/r4_bench_stats.jsonl || exit 1
cat gpurun_out/r4_bench_stats.jsonl
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step 2>/dev/null > gpurun_out/r4_collection.json || exit 1
cat gpurun_out/r4_collection.json | cut -c1-400
timeout -k 10 300 python benchmarks/bench_map.py 2>/dev/null > gpurun_out/r4_bench_map.json || exit 1
cat gpurun_out/r4_bench_map.json | cut -c1-400
timeout -k 10 300 python benchmarks/bench_gemm.py 2>/dev/null > gpurun_out/r4_bench_gemm.jsonl || exit 1
cat gpurun_out/r4_bench_gemm.jsonl | cut -c1-300
timeout -k 10 120 python benchmarks/bench_word_read.py 2>/dev/null > gpurun_out/r4_word_read.jsonl || exit 1
cat gpurun_out/r4_word_read.jsonl
