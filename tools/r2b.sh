# oneshot kernel tests + headline diagnostics + kernel-only stats at HBM-streaming ring
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_oneshot_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2b_oneshot.log 2>&1; rc=$?; tail -25 gpurun_out/r2b_oneshot.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_headline_diag.py --rings 64,400 > gpurun_out/r2b_diag.jsonl 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r2b_diag.jsonl; [ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_diag -o p --output-format csv -- python3 $R/benchmarks/bench_headline_diag.py --rings 400 > $R/gpurun_out/prof_diag.log 2>&1) || { tail -20 gpurun_out/prof_diag.log; exit 1; }
f=$(find gpurun_out/prof_diag -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r2b_diag_kernel_stats.csv; rm -rf gpurun_out/prof_diag
cut -d, -f1-4 gpurun_out/r2b_diag_kernel_stats.csv | head -6
