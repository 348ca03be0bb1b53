#!/bin/bash
# Round 5: the library rebuilt with kernarg preload; headline command x5, reset() variants of the first region,
# a 200-step kernel trace of the headline, and the native roctx ranges around the production update.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
for i in 1 2 3 4 5; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5p_b20_$i.log 2>&1 || { tail -20 gpurun_out/r5p_b20_$i.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/r5p_b20_$i.log
done
for c in onering onering_zero onering onering_zero onering onering_zero; do
  timeout -k 10 120 python3 benchmarks/first_region_probe.py $c >> gpurun_out/r5_first_region3.jsonl 2>gpurun_out/r5_fr3.err || { tail -5 gpurun_out/r5_fr3.err; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r5_first_region3.jsonl"):
    d = json.loads(l)
    print(d["case"], d.get("reset_us"), d["rep0"], d["rep1"], "host0", d["per_update0"][:8])
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5p_prof -o p -- python3 $R/bench.py --steps 200 --warmup 20 --no-baseline > $R/gpurun_out/r5p_prof.log 2>&1 || { tail -20 $R/gpurun_out/r5p_prof.log; exit 1; }
cd $R && python3 tools/gpu/trace_summary.py gpurun_out/r5p_prof --match mc_argmax
cd /tmp && TORCHMETRICS_AMD_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $R/gpurun_out/r5p_marker -o m -- python3 $R/bench.py --steps 20 --warmup 5 --no-baseline > $R/gpurun_out/r5p_marker.log 2>&1 || { tail -20 $R/gpurun_out/r5p_marker.log; exit 1; }
cd $R && ls gpurun_out/r5p_marker/*/ 2>/dev/null | head; find gpurun_out/r5p_marker -name "*marker*" | head
