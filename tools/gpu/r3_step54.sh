#!/bin/bash
# final-build traces: headline kernel stats (ours only), config #5 eager compute every step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final -o ours -- python3 $R/bench.py --steps 200 --warmup 20 --no-baseline > $R/gpurun_out/r3_prof_final.log 2>&1 || { tail -20 $R/gpurun_out/r3_prof_final.log; exit 1; }
cd $R && cp $(find gpurun_out/prof_final -name "*kernel_stats.csv" | head -1) gpurun_out/r3_headline_ours_kernel_stats_final.csv && rm -rf gpurun_out/prof_final
cut -d, -f1-4 gpurun_out/r3_headline_ours_kernel_stats_final.csv | cut -c1-140 | head -5
grep metric gpurun_out/r3_prof_final.log | cut -c1-200
timeout -k 10 300 python benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step 2>/dev/null > gpurun_out/r3_collection_sync_every_step_final.json || exit 1
cut -c1-200 gpurun_out/r3_collection_sync_every_step_final.json
