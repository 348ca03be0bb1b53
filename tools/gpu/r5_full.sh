#!/bin/bash
# Round-5 full GPU suite + smoke + two headline runs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5f_pytest_gpu.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5f_pytest_gpu.log | tail -30
[[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f_smoke.log 2>&1 || { tail -30 gpurun_out/r5f_smoke.log; exit 1; }
tail -1 gpurun_out/r5f_smoke.log
for i in 1 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5f_bench20_$i.log 2>&1 || { tail -30 gpurun_out/r5f_bench20_$i.log; exit 1; }
  grep '^{' gpurun_out/r5f_bench20_$i.log | cut -c1-200
done
