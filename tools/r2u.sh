#!/bin/bash
# Final re-entry GPU pass: the new kernels' tests + bench + rocprof (tools/r2t.sh), then the whole -m gpu suite,
# smoke() and bench.py with the driver's arguments.  Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
bash tools/r2t.sh || exit $?
cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/full_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/full_gpu.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" gpurun_out/full_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_20.json 2> gpurun_out/bench_20.err || { tail -20 gpurun_out/bench_20.err; exit 1; }
cat gpurun_out/bench_20.json
