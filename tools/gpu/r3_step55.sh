#!/bin/bash
# A/B of the few-bin LDS staging on config #5 (update only and compute every step), same box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
: > gpurun_out/r3_fewbins_ab.jsonl
for rep in 1 2; do
  for st in 1 0; do
    TM_AMD_FEWBINS_STAGE=$st timeout -k 10 200 python benchmarks/bench_collection.py --steps 300 --warmup 30 --no-baseline 2>/dev/null | sed "s/^/{\"stage\": $st, \"mode\": \"update\", \"r\": /; s/$/}/" >> gpurun_out/r3_fewbins_ab.jsonl || exit 1
    TM_AMD_FEWBINS_STAGE=$st timeout -k 10 200 python benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step --no-baseline 2>/dev/null | sed "s/^/{\"stage\": $st, \"mode\": \"compute\", \"r\": /; s/$/}/" >> gpurun_out/r3_fewbins_ab.jsonl || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3_fewbins_ab.jsonl"):
    d = json.loads(l); print(d["stage"], d["mode"], d["r"]["ms_per_step"])
PY
