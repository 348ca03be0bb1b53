#!/bin/bash
# window-stat kernels, classification/confmat regression after the 512-thread ord16 launch, headline 20-step x3,
# and the HIP scheduling-mode probe
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
bash tools/gpu/tests.sh step10_tests tests/test_window_stats_gpu.py tests/test_native_update.py tests/test_kernels_gpu.py || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_s10_bench20_$i.log 2>&1 || { tail -30 gpurun_out/r3_s10_bench20_$i.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/r3_s10_bench20_$i.log | head -1
done
rm -f gpurun_out/r3_first_region2.jsonl
for case in plain sched_spin sched_yield plain sched_spin sched_yield; do
  timeout -k 10 120 python -u benchmarks/first_region_probe.py $case 2>/dev/null >> gpurun_out/r3_first_region2.jsonl || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/r3_first_region2.jsonl'):
    d = json.loads(l); print(d['case'], d['rep0'], d['rep1'], d['rep2'])
"
