#!/bin/bash
# Round-5 attributable kernel traces: each benchmark in an ours-only mode (no emulated reference, no parity solver in
# the same process), rocprofv3 --kernel-trace --stats; the *_kernel_stats.csv files land in gpurun_out/r5prof_*.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
prof() {  # name, then the python script and its args
  local name=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$name -o p -- python3 "$@" > $R/gpurun_out/r5prof_$name.log 2>&1 || { tail -20 $R/gpurun_out/r5prof_$name.log; return 1; }
  cd $R && cp $(find gpurun_out/prof_$name -name "*kernel_stats.csv" | head -1) gpurun_out/r5prof_${name}_kernel_stats.csv && rm -rf gpurun_out/prof_$name
  echo "== $name"; cut -d, -f1-4 gpurun_out/r5prof_${name}_kernel_stats.csv | cut -c1-160 | head -8
}
prof headline $R/bench.py --steps 200 --warmup 20 --no-baseline || exit 1
prof clustering $R/benchmarks/bench_clustering.py --ours-only || exit 1
prof stats $R/benchmarks/bench_binary_stats.py || exit 1
prof forward $R/benchmarks/bench_forward.py || exit 1
prof gemm16 $R/benchmarks/gemm16_one.py --iters 20 || exit 1
# roctx ranges on the production path: the native entry points' ranges around their kernels
cd /tmp && TORCHMETRICS_AMD_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $R/gpurun_out/prof_markers -o p -- python3 $R/benchmarks/bench_forward.py > $R/gpurun_out/r5prof_markers.log 2>&1 || { tail -20 $R/gpurun_out/r5prof_markers.log; exit 1; }
cd $R && python3 tools/gpu/marker_summary.py gpurun_out/prof_markers > gpurun_out/r5prof_forward_markers.txt 2>&1; head -30 gpurun_out/r5prof_forward_markers.txt; rm -rf gpurun_out/prof_markers
