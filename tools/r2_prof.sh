# Round-2 profile pass: sort/scan + GEMM-family benches, each under rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for b in bench_sorted bench_gemm bench_kid; do
  timeout -k 10 300 python benchmarks/$b.py > gpurun_out/r02_$b.jsonl 2> gpurun_out/r02_$b.err || { tail -30 gpurun_out/r02_$b.err; exit 1; }
  cat gpurun_out/r02_$b.jsonl
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$b -o p --output-format csv -- python3 $R/benchmarks/$b.py > $R/gpurun_out/prof_$b.log 2>&1) || { tail -30 gpurun_out/prof_$b.log; exit 1; }
  f=$(find gpurun_out/prof_$b -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r02_${b}_kernel_stats.csv; rm -rf gpurun_out/prof_$b
  cut -d, -f1-4 gpurun_out/r02_${b}_kernel_stats.csv | head -12
done
