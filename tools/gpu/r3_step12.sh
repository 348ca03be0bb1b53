#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
rm -f gpurun_out/r3_first_region3.jsonl
for case in onering onering_read onering_heavy onering onering_read onering_heavy; do
  timeout -k 10 120 python -u benchmarks/first_region_probe.py $case 2>/dev/null >> gpurun_out/r3_first_region3.jsonl || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/r3_first_region3.jsonl'):
    d = json.loads(l); print(d['case'], d['rep0'], d['rep1'], d['rep2'])
"
