#!/bin/bash
# Round 5: (1) the headline under host-memory kernel arguments (the library's kernels are kernarg-preloaded);
# (2) compute()'s completion-check variants on the standalone region; (3) marker + runtime + kernel trace of the
# production update with ranges on; (4) the new GPU tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
for i in 1 2 3 4 5; do
  HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-baseline > gpurun_out/r5t_b20_$i.log 2>&1 || { tail -20 gpurun_out/r5t_b20_$i.log; exit 1; }
  echo "hostkarg $(grep -o '"value": [0-9.]*' gpurun_out/r5t_b20_$i.log)"
done
for mode in memcpy streamsync eventsync none memcpy streamsync eventsync none; do
  timeout -k 10 60 tools/mb/region_mb_pre pre $mode >> gpurun_out/r5_region_tail.jsonl 2>&1 || exit 1
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r5_region_tail.jsonl"):
    d = json.loads(l)
    print(d["compute_mode"], "steady", d["steady_us_per_launch"], *[d[f"rep{r}"] for r in range(4)])
PY
cd /tmp && TORCHMETRICS_AMD_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --hip-runtime-trace --kernel-trace --output-format csv -d $R/gpurun_out/r5t_marker -o m -- python3 $R/bench.py --steps 20 --warmup 5 --no-baseline > $R/gpurun_out/r5t_marker.log 2>&1 || { tail -20 $R/gpurun_out/r5t_marker.log; exit 1; }
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_native_update.py tests/test_profiling.py tests/test_native_forward_gpu.py -m gpu > gpurun_out/r5t_tests.log 2>&1 || { tail -30 gpurun_out/r5t_tests.log; exit 1; }
tail -2 gpurun_out/r5t_tests.log
