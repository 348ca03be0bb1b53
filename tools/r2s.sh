#!/bin/bash
# Re-entry GPU pass: new aggregation kernel tests first, then the whole -m gpu suite, smoke(), bench.py (driver
# arguments) and the aggregation bench.  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_aggregation_gpu.py tests/test_exact_match_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/agg_gpu.log 2>&1 || { tail -40 gpurun_out/agg_gpu.log; exit 1; }
tail -2 gpurun_out/agg_gpu.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/full_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/full_gpu.log | grep -v "^\.\.\." 
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_20.json 2> gpurun_out/bench_20.err || { tail -20 gpurun_out/bench_20.err; exit 1; }
cat gpurun_out/bench_20.json
timeout -k 10 300 python -u benchmarks/bench_aggregation.py > gpurun_out/bench_agg.jsonl 2> gpurun_out/bench_agg.err || { tail -20 gpurun_out/bench_agg.err; exit 1; }
cat gpurun_out/bench_agg.jsonl
