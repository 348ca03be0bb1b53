#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fused_update_gpu.py tests/test_calibration_cache_gpu.py tests/test_fused_compute_gpu.py -m gpu > gpurun_out/r5f6_tests.log 2>&1 || { grep -E "^FAILED|^ERROR|Error|assert|passed|failed" gpurun_out/r5f6_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r5f6_tests.log
cd /tmp
for ab in 0 2; do
  TM_AMD_FAMILY_ABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fp3 -o p -- python3 $R/benchmarks/family_probe.py > $R/gpurun_out/fp3.log 2>&1 || { tail -5 $R/gpurun_out/fp3.log; exit 1; }
  echo "ablate=$ab $(grep step_us $R/gpurun_out/fp3.log | cut -c1-60) $(python3 $R/tools/gpu/kstats.py $R/gpurun_out/fp3 family_rows | cut -c73-)"
  rm -rf $R/gpurun_out/fp3
done
