#!/bin/bash
# Session re-entry check: retrieval PR-curve kernel tests, full GPU suite, smoke, three 20-step headline runs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_retrieval_kernel.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_retrieval_gpu.log 2>&1 || { tail -30 gpurun_out/r3_retrieval_gpu.log; exit 1; }
tail -1 gpurun_out/r3_retrieval_gpu.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_full_gpu_suite.log 2>&1
rc=$?
tail -8 gpurun_out/r3_full_gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench20_$i.json 2> gpurun_out/r3_bench20_$i.err || { tail -20 gpurun_out/r3_bench20_$i.err; exit 1; }
  cut -c1-160 gpurun_out/r3_bench20_$i.json
done
