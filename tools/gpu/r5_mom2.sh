#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_regression.py tests/test_fused_compute_gpu.py tests/test_stream_kernels_gpu.py tests/test_kernels_gpu.py tests/test_corr_merge.py tests/test_kernel_boundaries_gpu.py -m gpu > gpurun_out/r5m2_tests.log 2>&1 || { tail -30 gpurun_out/r5m2_tests.log; exit 1; }
tail -1 gpurun_out/r5m2_tests.log
for h in 1 0 8192; do
  TM_AMD_MOMENTS_HANDOFF=$h timeout -k 10 200 python3 benchmarks/moments_probe.py > gpurun_out/r5m2_probe_$h.jsonl 2>&1 || { tail -5 gpurun_out/r5m2_probe_$h.jsonl; exit 1; }
  echo "handoff=$h"; grep '"n"' gpurun_out/r5m2_probe_$h.jsonl
done
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/m2 -o p -- python3 $R/benchmarks/moments_probe.py --n 1024 8192 65536 --cases config5 > $R/gpurun_out/m2.log 2>&1 || { tail -5 $R/gpurun_out/m2.log; exit 1; }
cd $R && python3 tools/gpu/kstats.py gpurun_out/m2 moments; rm -rf gpurun_out/m2
timeout -k 10 300 python3 benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 > gpurun_out/r5m2_sync.json 2>&1 || { tail -5 gpurun_out/r5m2_sync.json; exit 1; }
tail -1 gpurun_out/r5m2_sync.json | cut -c1-200; tail -1 gpurun_out/r5m2_sync.json | grep -o '"phases_ms_per_step_max_over_ranks": {[^}]*}'
