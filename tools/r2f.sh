set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $R/gpurun_out/prof_f -o p --output-format csv -- python3 $R/benchmarks/bench_collection.py --steps 200 --warmup 10 --sync-every-step --graph > $R/gpurun_out/prof_f.log 2>&1) || { tail -20 gpurun_out/prof_f.log; exit 1; }
for f in $(find gpurun_out/prof_f -name "*_stats.csv"); do cp $f gpurun_out/r2f_$(basename $f); done
f=$(find gpurun_out/prof_f -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/r2f_kernel_trace.csv
rm -rf gpurun_out/prof_f
ls gpurun_out/ | grep r2f
cut -d, -f1-4 gpurun_out/r2f_p_kernel_stats.csv | cut -c1-150 | head -30
cut -d, -f1-4 gpurun_out/r2f_p_hip_api_stats.csv | head -25
