#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fused_update_gpu.py tests/test_fused_compute_gpu.py -m gpu > gpurun_out/r5fp2_tests.log 2>&1 || { tail -30 gpurun_out/r5fp2_tests.log; exit 1; }
tail -1 gpurun_out/r5fp2_tests.log
cd /tmp
for cfg in "1 128" "1 256" "1 512"; do
  set -- $cfg
  TM_AMD_FAMILY_G=$1 TM_AMD_FAMILY_BLOCKS=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fp2 -o p -- python3 $R/benchmarks/family_probe.py > $R/gpurun_out/fp2.log 2>&1 || { tail -5 $R/gpurun_out/fp2.log; exit 1; }
  echo "G=$1 blocks=$2 $(grep step_us $R/gpurun_out/fp2.log)"
  python3 $R/tools/gpu/kstats.py $R/gpurun_out/fp2 family moments
  rm -rf $R/gpurun_out/fp2
done
