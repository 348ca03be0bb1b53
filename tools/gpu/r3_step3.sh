#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u benchmarks/cold_region_probe.py > gpurun_out/r3_cold_region.json 2>gpurun_out/r3_cold_region.err || { tail -20 gpurun_out/r3_cold_region.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r3_cold_region.json'))
for k,v in d.items():
    for run in v:
        for r in run: print(k, r)
"
