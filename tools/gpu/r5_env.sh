#!/bin/bash
# Round 5: the first timed region under HIP runtime settings -- the standalone region microbenchmark (no Python) and
# the driver's bench command, fresh processes per case.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
MB=tools/mb/region_mb
run_mb() {  # label, env assignments...
  local label=$1; shift
  for i in 1 2; do env "$@" timeout -k 10 60 $MB $label >> gpurun_out/r5_region_mb.jsonl 2>&1 || { echo "mb $label failed"; return 1; }; done
}
run_mb default || exit 1
run_mb awt0 ROC_ACTIVE_WAIT_TIMEOUT=0 || exit 1
run_mb awt1000 ROC_ACTIVE_WAIT_TIMEOUT=1000 || exit 1
run_mb devkarg0 HIP_FORCE_DEV_KERNARG=0 || exit 1
run_mb devkarg1 HIP_FORCE_DEV_KERNARG=1 || exit 1
run_mb nointr HSA_ENABLE_INTERRUPT=0 || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r5_region_mb.jsonl"):
    try:
        d = json.loads(l)
    except Exception:
        print(l[:200]); continue
    print(d["case"], *[d[f"rep{r}"] for r in range(4)])
PY
bench() {  # label, env...
  local label=$1; shift
  for i in 1 2 3; do
    env "$@" timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-baseline > gpurun_out/r5_env_$label_$i.log 2>&1 || { tail -5 gpurun_out/r5_env_$label_$i.log; return 1; }
    echo "$label $(grep -o '"value": [0-9.]*' gpurun_out/r5_env_$label_$i.log)"
  done
}
bench default || exit 1
bench awt1000 ROC_ACTIVE_WAIT_TIMEOUT=1000 || exit 1
bench nointr HSA_ENABLE_INTERRUPT=0 || exit 1
bench devkarg0 HIP_FORCE_DEV_KERNARG=0 || exit 1
