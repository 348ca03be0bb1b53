#!/bin/bash
# GPU step: the whole -m gpu suite (as the driver runs it) + smoke() + a 1-GPU bench.py run
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH="$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/full_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/full_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; cat gpurun_out/bench_default.json; exit $rc
