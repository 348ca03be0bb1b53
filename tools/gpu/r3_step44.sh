#!/bin/bash
# Full GPU suite + smoke after the stats-count / setattr / forward changes; forward and headline benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_full_gpu_suite.log 2>&1
rc=$?
tail -3 gpurun_out/r3_full_gpu_suite.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/r3_full_gpu_suite.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
timeout -k 10 300 python benchmarks/bench_forward.py > gpurun_out/r3_bench_forward.jsonl 2>gpurun_out/r3_bench_forward.err || { tail -20 gpurun_out/r3_bench_forward.err; exit 1; }
cat gpurun_out/r3_bench_forward.jsonl
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench20_$i.json 2> gpurun_out/r3_bench20_$i.err || { tail -20 gpurun_out/r3_bench20_$i.err; exit 1; }
  cut -c1-120 gpurun_out/r3_bench20_$i.json
done
