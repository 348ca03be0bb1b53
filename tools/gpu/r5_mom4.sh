#!/bin/bash
# moments kernels: per-kernel device time by size (config #5 plan), single block vs hand-off
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_regression.py tests/test_fused_compute_gpu.py tests/test_kernels_gpu.py tests/test_fused_misc_gpu.py tests/test_corr_merge.py tests/test_kernel_boundaries_gpu.py tests/test_fused_update_gpu.py -m gpu > gpurun_out/r5m4_tests.log 2>&1 || { tail -30 gpurun_out/r5m4_tests.log; exit 1; }
tail -1 gpurun_out/r5m4_tests.log
for n in 1024 8192 65536 262144; do for h in 8192 0; do
cd /tmp && TM_AMD_MOMENTS_HANDOFF=$h timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/m3 -o p -- python3 $R/benchmarks/moments_probe.py --n $n --cases config5 > $R/gpurun_out/m3.log 2>&1 || { tail -5 $R/gpurun_out/m3.log; exit 1; }
cd $R && echo "n=$n handoff=$h" >> gpurun_out/r5m4_kstats.txt && python3 tools/gpu/kstats.py gpurun_out/m3 moments >> gpurun_out/r5m4_kstats.txt; rm -rf gpurun_out/m3
done; done
cat gpurun_out/r5m4_kstats.txt
