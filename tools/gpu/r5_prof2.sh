#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_clustering_gpu.py tests/test_clustering.py -m gpu > gpurun_out/r5p2_tests.log 2>&1 || { tail -30 gpurun_out/r5p2_tests.log; exit 1; }
tail -1 gpurun_out/r5p2_tests.log
prof() {
  local name=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$name -o p -- python3 "$@" > $R/gpurun_out/r5prof_$name.log 2>&1 || { tail -20 $R/gpurun_out/r5prof_$name.log; return 1; }
  cd $R && cp $(find gpurun_out/prof_$name -name "*kernel_stats.csv" | head -1) gpurun_out/r5prof_${name}_kernel_stats.csv && rm -rf gpurun_out/prof_$name
  echo "== $name"
}
prof clustering $R/benchmarks/bench_clustering.py --ours-only || exit 1
prof forward $R/benchmarks/bench_forward.py --ours-only || exit 1
grep '^{' gpurun_out/r5prof_clustering.log | cut -c1-300
grep '^{' gpurun_out/r5prof_forward.log | cut -c1-300
cd /tmp && TORCHMETRICS_AMD_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --hip-runtime-trace --kernel-trace --output-format csv -d $R/gpurun_out/prof_markers -o p -- python3 $R/benchmarks/bench_forward.py --ours-only --steps 50 > $R/gpurun_out/r5prof_markers.log 2>&1 || { tail -20 $R/gpurun_out/r5prof_markers.log; exit 1; }
cd $R && python3 tools/gpu/marker_summary.py gpurun_out/prof_markers > gpurun_out/r5prof_forward_markers.txt 2>&1; head -30 gpurun_out/r5prof_forward_markers.txt; rm -rf gpurun_out/prof_markers
