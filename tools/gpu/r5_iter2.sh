#!/bin/bash
# Round 5 iteration 2: G-lanes-per-row family kernel (A/B vs one row per thread, block caps), 512-thread moments block.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fused_update_gpu.py tests/test_fused_compute_gpu.py tests/test_regression.py -m gpu > gpurun_out/r5i2_tests.log 2>&1 || { tail -40 gpurun_out/r5i2_tests.log; exit 1; }
tail -1 gpurun_out/r5i2_tests.log
timeout -k 10 200 python3 benchmarks/moments_probe.py > gpurun_out/r5i2_moments.jsonl 2>&1 || { tail -5 gpurun_out/r5i2_moments.jsonl; exit 1; }
grep '"n"' gpurun_out/r5i2_moments.jsonl
for cfg in "1 128" "1 64" "1 256" "0 512"; do
  set -- $cfg
  TM_AMD_FAMILY_G=$1 TM_AMD_FAMILY_BLOCKS=$2 timeout -k 10 300 python3 benchmarks/bench_collection.py --steps 200 --warmup 20 --no-baseline > gpurun_out/r5i2_coll_upd_$1_$2.json 2>&1 || { tail -5 gpurun_out/r5i2_coll_upd_$1_$2.json; exit 1; }
  echo "G=$1 blocks=$2: $(tail -1 gpurun_out/r5i2_coll_upd_$1_$2.json | cut -c1-330)"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5i2_prof -o p -- python3 $R/benchmarks/bench_collection.py --sync-every-step --steps 100 --warmup 10 --no-baseline > $R/gpurun_out/r5i2_prof.log 2>&1 || { tail -20 $R/gpurun_out/r5i2_prof.log; exit 1; }
cd $R && python3 tools/gpu/trace_summary.py gpurun_out/r5i2_prof --calls 110 > gpurun_out/r5i2_trace_summary.txt; head -12 gpurun_out/r5i2_trace_summary.txt; tail -1 gpurun_out/r5i2_trace_summary.txt; rm -rf gpurun_out/r5i2_prof
timeout -k 10 300 python3 benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 > gpurun_out/r5i2_coll_sync.json 2>&1 || { tail -5 gpurun_out/r5i2_coll_sync.json; exit 1; }
tail -1 gpurun_out/r5i2_coll_sync.json | cut -c1-900
for w in cls reg; do
  timeout -k 10 200 python3 benchmarks/compute_cprofile.py --which $w > gpurun_out/r5i2_cprof_$w.txt 2>&1 || { tail -5 gpurun_out/r5i2_cprof_$w.txt; exit 1; }
  timeout -k 10 200 python3 benchmarks/compute_cprofile.py --which $w --update-only > gpurun_out/r5i2_cprof_${w}_upd.txt 2>&1 || { tail -5 gpurun_out/r5i2_cprof_${w}_upd.txt; exit 1; }
done
grep -m3 "function calls" gpurun_out/r5i2_cprof_*.txt
