#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/mb/confmat_ring_mb > gpurun_out/r3_confmat_ring_mb2.jsonl 2>&1 || { tail -20 gpurun_out/r3_confmat_ring_mb2.jsonl; exit 1; }
cat gpurun_out/r3_confmat_ring_mb2.jsonl
bash tools/gpu/tests.sh clustering_tests tests/test_clustering_gpu.py || exit 1
timeout -k 10 300 python -u benchmarks/bench_clustering.py > gpurun_out/r3_bench_clustering.jsonl 2> gpurun_out/r3_bench_clustering.err || { tail -20 gpurun_out/r3_bench_clustering.err; exit 1; }
cat gpurun_out/r3_bench_clustering.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_cl -o cl -- python3 $R/benchmarks/bench_clustering.py > $R/gpurun_out/r3_prof_cl.log 2>&1 || { tail -20 $R/gpurun_out/r3_prof_cl.log; exit 1; }
cd $R && cp $(find gpurun_out/prof_cl -name "*kernel_stats.csv" | head -1) gpurun_out/r3_clustering_kernel_stats.csv && rm -rf gpurun_out/prof_cl
cut -d, -f1-4 gpurun_out/r3_clustering_kernel_stats.csv | head -14
