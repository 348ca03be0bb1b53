#!/bin/bash
# Round-5 re-measure after the wave-reduction change: config #5 (sync-every-step, update-only, ours-only device
# trace), the stat-score update bench, the native forward, the headline kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=gpurun_out/r5meas.txt
: > $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_bin_fused_finalize_gpu.py tests/test_regression.py tests/test_kernels_gpu.py tests/test_fused_update_gpu.py -m gpu > gpurun_out/r5meas_tests.log 2>&1 || { tail -30 gpurun_out/r5meas_tests.log; exit 1; }
tail -1 gpurun_out/r5meas_tests.log >> $O
for i in 1 2; do
timeout -k 10 300 python3 benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 > gpurun_out/r5meas_sync_$i.json 2>&1 || { tail -5 gpurun_out/r5meas_sync_$i.json; exit 1; }
tail -1 gpurun_out/r5meas_sync_$i.json | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"phases_ms_per_step_max_over_ranks": {[^}]*}' >> $O
done
timeout -k 10 300 python3 benchmarks/bench_collection.py --steps 200 --warmup 20 > gpurun_out/r5meas_upd.json 2>&1 || { tail -5 gpurun_out/r5meas_upd.json; exit 1; }
echo "update-only:" >> $O; tail -1 gpurun_out/r5meas_upd.json | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' >> $O
timeout -k 10 200 python3 benchmarks/bench_binary_stats.py > gpurun_out/r5meas_stats.jsonl 2>&1 || { tail -5 gpurun_out/r5meas_stats.jsonl; exit 1; }
cut -c1-220 gpurun_out/r5meas_stats.jsonl >> $O
timeout -k 10 200 python3 benchmarks/bench_forward.py --ours-only > gpurun_out/r5meas_fwd.jsonl 2>&1 || { tail -5 gpurun_out/r5meas_fwd.jsonl; exit 1; }
cat gpurun_out/r5meas_fwd.jsonl >> $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pc -o p -- python3 $R/benchmarks/bench_collection.py --sync-every-step --steps 200 --warmup 20 --no-baseline > $R/gpurun_out/pc.log 2>&1 || { tail -5 $R/gpurun_out/pc.log; exit 1; }
cd $R && cp $(find gpurun_out/pc -name "*kernel_stats.csv" | head -1) gpurun_out/r5meas_collection_sync_kernel_stats.csv && echo "collection sync ours-only kernels:" >> $O && python3 tools/gpu/kstats.py gpurun_out/pc "" | head -25 >> $O; rm -rf gpurun_out/pc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ps -o p -- python3 $R/benchmarks/bench_binary_stats.py > $R/gpurun_out/ps.log 2>&1 || { tail -5 $R/gpurun_out/ps.log; exit 1; }
cd $R && cp $(find gpurun_out/ps -name "*kernel_stats.csv" | head -1) gpurun_out/r5meas_stats_kernel_stats.csv && echo "stats kernels:" >> $O && python3 tools/gpu/kstats.py gpurun_out/ps "" | head -25 >> $O; rm -rf gpurun_out/ps
cat $O
