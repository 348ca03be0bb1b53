#!/bin/bash
# One-shot fail-safe + native update: targeted GPU tests, then host-side update cost and three short headline runs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
bash tools/gpu/tests.sh step1_tests tests/test_native_update.py tests/test_oneshot_gpu.py tests/test_exact_match_gpu.py tests/test_calibration_cache_gpu.py || exit 1
timeout -k 10 300 python -u benchmarks/host_update_profile.py > gpurun_out/r3_host_profile2.log 2>&1 || { tail -30 gpurun_out/r3_host_profile2.log; exit 1; }
head -3 gpurun_out/r3_host_profile2.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_s1_bench20_$i.log 2>&1 || { tail -30 gpurun_out/r3_s1_bench20_$i.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/r3_s1_bench20_$i.log | head -1
done
