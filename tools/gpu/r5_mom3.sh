#!/bin/bash
# moments small-kernel tail (prefetched destinations) + family fold atomics: tests, probe, kernel stats, collection
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_regression.py tests/test_fused_compute_gpu.py tests/test_stream_kernels_gpu.py tests/test_kernels_gpu.py tests/test_corr_merge.py tests/test_kernel_boundaries_gpu.py tests/test_fused_update_gpu.py tests/test_collection_checks_gpu.py tests/test_fused_misc_gpu.py -m gpu > gpurun_out/r5m3_tests.log 2>&1 || { tail -30 gpurun_out/r5m3_tests.log; exit 1; }
tail -1 gpurun_out/r5m3_tests.log
for h in 1 0 8192; do
  TM_AMD_MOMENTS_HANDOFF=$h timeout -k 10 200 python3 benchmarks/moments_probe.py > gpurun_out/r5m3_probe_$h.jsonl 2>&1 || { tail -5 gpurun_out/r5m3_probe_$h.jsonl; exit 1; }
  echo "handoff=$h"; grep '"n"' gpurun_out/r5m3_probe_$h.jsonl
done
for h in 1 0; do
cd /tmp && TM_AMD_MOMENTS_HANDOFF=$h timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/m3 -o p -- python3 $R/benchmarks/moments_probe.py --n 1024 8192 65536 --cases config5 > $R/gpurun_out/m3.log 2>&1 || { tail -5 $R/gpurun_out/m3.log; exit 1; }
cd $R && echo "handoff=$h" && python3 tools/gpu/kstats.py gpurun_out/m3 moments; rm -rf gpurun_out/m3
done
timeout -k 10 300 python3 benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 > gpurun_out/r5m3_sync.json 2>&1 || { tail -5 gpurun_out/r5m3_sync.json; exit 1; }
tail -1 gpurun_out/r5m3_sync.json | cut -c1-200; tail -1 gpurun_out/r5m3_sync.json | grep -o '"phases_ms_per_step_max_over_ranks": {[^}]*}'
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/m4 -o p -- python3 $R/benchmarks/bench_collection.py --sync-every-step --steps 100 --warmup 10 > $R/gpurun_out/m4.log 2>&1 || { tail -5 $R/gpurun_out/m4.log; exit 1; }
cd $R && python3 tools/gpu/kstats.py gpurun_out/m4 ""; rm -rf gpurun_out/m4
