set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python benchmarks/graphed_compute_breakdown.py 2>&1 | grep -v amdgpu.ids || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gc -o p --output-format csv -- python3 $R/benchmarks/bench_collection.py --steps 100 --warmup 10 --sync-every-step --graph > $R/gpurun_out/prof_gc.log 2>&1) || { tail -20 gpurun_out/prof_gc.log; exit 1; }
f=$(find gpurun_out/prof_gc -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r2d_gc_kernel_stats.csv; rm -rf gpurun_out/prof_gc
cut -d, -f1-4 gpurun_out/r2d_gc_kernel_stats.csv | cut -c1-160 | head -40
