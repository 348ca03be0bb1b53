#!/bin/bash
# Exact-match vector kernel check + headline variance probe (bench.py at the driver's arguments, twice, and 200 steps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_exact_match_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/em_gpu.log 2>&1 || { tail -40 gpurun_out/em_gpu.log; exit 1; }
tail -1 gpurun_out/em_gpu.log
timeout -k 10 300 python -u benchmarks/bench_aggregation.py > gpurun_out/bench_agg.jsonl 2> gpurun_out/bench_agg.err || { tail -20 gpurun_out/bench_agg.err; exit 1; }
cat gpurun_out/bench_agg.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_20_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_20_$i.json'));print('steps20', d['value'], d['ms_per_step'], d['compute_ms'])"
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_200.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_200.json'));print('steps200', d['value'], d['ms_per_step'], d['compute_ms'], d['vs_baseline'])"
