#!/bin/bash
# Round-4 first GPU call: full GPU suite, smoke, two fresh 20-step headline runs, forward / stat-score update / config #5
# benches (baselines for this round's work).  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_native_forward_gpu.py tests/test_native_update.py tests/test_stream_kernels_gpu.py tests/test_macro_curves.py tests/test_iou_module.py tests/test_fused_compute_gpu.py tests/test_functional_kernels_gpu.py tests/test_torchscript.py tests/test_audio.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pytest_fwd.log 2>&1 || { tail -60 gpurun_out/r4_pytest_fwd.log; exit 1; }
tail -2 gpurun_out/r4_pytest_fwd.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r4_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -30 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench20_$i.log 2>&1 || { tail -30 gpurun_out/r4_bench20_$i.log; exit 1; }
  grep '^{' gpurun_out/r4_bench20_$i.log | cut -c1-200
done
timeout -k 10 300 python benchmarks/bench_forward.py 2>/dev/null > gpurun_out/r4_bench_forward.jsonl || exit 1
cat gpurun_out/r4_bench_forward.jsonl
timeout -k 10 300 python benchmarks/bench_binary_stats.py 2>/dev/null > gpurun_out/r4_bench_stats.jsonl || exit 1
cat gpurun_out/r4_bench_stats.jsonl
timeout -k 10 300 python benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step 2>/dev/null > gpurun_out/r4_collection_before.json || exit 1
cat gpurun_out/r4_collection_before.json
