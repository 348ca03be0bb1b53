# config #5 profiles: graphed step phases + kernel stats of the graphed per-step-compute bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step --graph > gpurun_out/r02_collection_bench.jsonl 2>&1 || exit 1
timeout -k 10 200 python benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step >> gpurun_out/r02_collection_bench.jsonl 2>&1 || exit 1
timeout -k 10 200 python benchmarks/bench_collection.py --steps 300 --warmup 30 --graph >> gpurun_out/r02_collection_bench.jsonl 2>&1 || exit 1
timeout -k 10 200 python benchmarks/bench_collection.py --steps 300 --warmup 30 >> gpurun_out/r02_collection_bench.jsonl 2>&1 || exit 1
grep -v amdgpu gpurun_out/r02_collection_bench.jsonl
timeout -k 10 200 python benchmarks/graphed_compute_breakdown.py > gpurun_out/r02_graphed_compute_breakdown.json 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c -o p --output-format csv -- python3 $R/benchmarks/bench_collection.py --steps 300 --warmup 30 --sync-every-step --graph > $R/gpurun_out/prof_c.log 2>&1) || { tail -20 gpurun_out/prof_c.log; exit 1; }
f=$(find gpurun_out/prof_c -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r02_collection_graphed_kernel_stats.csv; rm -rf gpurun_out/prof_c
echo done
